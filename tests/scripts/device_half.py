"""16-bit float collectives on HBM (bf16 / fp16, the extended dtype enum) over the direct
transport (ranks share the box's GPU; a 1 MiB stage buffer forces chunking).  The kernels
accumulate every element over all ranks in fp32 (rank order) and round once, so the expected
value is the fp32 sum of the rank inputs in rank order, rounded: compared bit for bit."""
import sys

import torch

import rabit_amd as rabit

rabit.init(sys.argv[1:], lib="standard", rabit_device=0, rabit_device_peer_buffer="1M",
           rabit_device_peer_timeout_sec=20)
rank, world = rabit.get_rank(), rabit.get_world_size()
dev = torch.device("cuda", 0)


def inputs(r, n, dt):
    g = torch.Generator().manual_seed(1000 * r + n)
    return torch.randn(n, generator=g).mul_(3).to(dt)


checked = 0
for dt in (torch.bfloat16, torch.float16):
    for n in (1, 7, 1000, 65536 + 3, (3 << 20) // 2 + 5):
        xs = [inputs(r, n, dt) for r in range(world)]
        for op in (rabit.SUM, rabit.MAX, rabit.MIN):
            t = xs[rank].to(dev)
            rabit.allreduce(t, op)
            if op == rabit.SUM:
                acc = xs[0].float()
                for r in range(1, world):
                    acc = acc + xs[r].float()
                want = acc.to(dt)
            else:
                st = torch.stack([x.float() for x in xs])
                want = (st.max(0).values if op == rabit.MAX else st.min(0).values).to(dt)
            assert torch.equal(t.cpu(), want), (dt, n, op, t[:4].cpu(), want[:4])
            checked += 1
        # gradient averaging: sum * (1/world) in fp32, rounded once
        t = xs[rank].to(dev)
        rabit.allreduce_prepared(t, t, rabit.SUM, rabit.PREP_SCALE, 1.0 / world)
        acc = xs[0].float()
        for r in range(1, world):
            acc = acc + xs[r].float()
        want = (acc * torch.tensor(1.0 / world, dtype=torch.float32)).to(dt)
        diff = (t.cpu().float() - want.float()).abs().max().item()
        assert diff <= 2 * torch.finfo(dt).eps * want.float().abs().max().item(), (dt, n, diff)
        checked += 1
rabit.set_error_mode(True)  # raise instead of ending the worker
try:
    rabit.allreduce(torch.ones(8, device=dev, dtype=torch.bfloat16), rabit.BITOR)
    raise SystemExit("BITOR accepted on bf16")
except Exception as e:  # noqa: BLE001
    assert "BitOR" in str(e) or "floating" in str(e), e
rabit.finalize()
print("[%d] HALF OK %d checks" % (rank, checked), flush=True)
