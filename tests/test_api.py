"""Python API semantics over several CPU ranks, for every library flavour."""
import os
import sys

import numpy as np
import pytest

from rabit_amd.launcher import LocalJob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tests", "scripts", "api_check.py")


@pytest.mark.parametrize("lib,extra", [("standard", []), ("base", []), ("mock", []),
                                      ("standard", ["rabit_elide_consensus=0"]),
                                      ("standard", ["rabit_reduce_ring_mincount=1"])])
@pytest.mark.parametrize("n", [1, 3])
def test_api_world(native_build, lib, extra, n):
    job = LocalJob([sys.executable, SCRIPT, lib] + extra, n, 1, capture=True, timeout=120,
                   print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-3000:]
    assert out.count("API OK") == n
    assert any("says hi" in m for m in job.tracker.messages)


def test_empty_engine_single_process(native_build):
    import rabit_amd as rabit

    rabit.init(lib="empty")
    try:
        assert rabit.get_world_size() == 1 and rabit.engine_name() == "empty"
        calls = []
        out = rabit.allreduce(np.ones(3), rabit.SUM, prepare_fun=lambda a: calls.append(1))
        assert calls == [1] and np.all(out == 1)
    finally:
        rabit.finalize()


def test_single_node_without_tracker(native_build):
    import rabit_amd as rabit

    rabit.init()
    try:
        assert rabit.get_rank() == 0 and rabit.get_world_size() == 1
        assert not rabit.is_distributed()
        assert rabit.broadcast("x", 0) == "x"
        v, _ = rabit.load_checkpoint()
        assert v == 0
        rabit.checkpoint({"a": 1})
        assert rabit.version_number() == 1
        # no direct transport without a GPU and peers: the link probe says so instead of failing
        assert rabit.link_probe(1 << 20) is None
        # the direct-transport knobs report "not up" rather than raising
        assert rabit.set_device_transport(rabit.TRANSPORT_DIRECT, "pipelined") is False
    finally:
        rabit.finalize()


def test_error_mode_raises(native_build):
    import rabit_amd as rabit

    rabit.init()
    rabit.set_error_mode(True)
    try:
        with pytest.raises(TypeError):
            rabit.allreduce(np.ones(2, dtype=np.int16), rabit.SUM)
        with pytest.raises(TypeError):
            rabit.allreduce(np.ones(2), rabit.BITOR)
    finally:
        rabit.finalize()


FUZZ = os.path.join(ROOT, "tests", "scripts", "fuzz_collectives.py")
FUZZ_PARAMS = {
    "default": [],
    "ring_small_buffer": ["rabit_reduce_ring_mincount=1", "rabit_reduce_buffer=4K"],
    "tree_pipelined": ["rabit_reduce_ring_mincount=1000000", "rabit_tree_reduce_minsize=1K",
                       "rabit_reduce_buffer=8K"],
    "shm_chunked": ["rabit_host_shm_min=1K", "rabit_host_shm_buffer=64K"],
    "tcp_only_no_elide": ["rabit_host_shm=0", "rabit_elide_consensus=0"],
}


@pytest.mark.parametrize("n", [2, 5])
@pytest.mark.parametrize("name", sorted(FUZZ_PARAMS))
def test_fuzz_collectives(native_build, name, n):
    """Random allreduce (4 ops x 8 dtypes), broadcast (random roots) and variable, wrapping
    allgather slices, sizes 0..300001 elements, exact against numpy, on every host algorithm
    (ring / pipelined tree / shared memory, buffers smaller than the messages)."""
    seed = 1000 + 17 * n + len(name)
    job = LocalJob([sys.executable, FUZZ, str(seed), "60"] + FUZZ_PARAMS[name], n, 1,
                   capture=True, timeout=180, print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-3000:]
    assert out.count("FUZZ OK") == n, out[-3000:]


def test_fuzz_collectives_with_failures(native_build):
    """The same random stream with three workers killed at different points (mock engine):
    restarted workers resume from the last checkpoint and replay, every result stays exact."""
    job = LocalJob([sys.executable, FUZZ, "5", "80", "lib=mock", "mock=1,2,3,0", "mock=3,4,0,0",
                    "mock=0,4,7,0"], 4, 3, capture=True, timeout=240, print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-3000:]
    assert out.count("FUZZ OK") == 4, out[-3000:]
    assert sum(a - 1 for a in job.attempts) == 3, job.attempts


@pytest.mark.parametrize("extra", [[], ["rabit_reduce_ring_mincount=1"]])
def test_half_precision_host(native_build, extra):
    """extended dtypes kHalf / kBFloat16 on the host path (tree and ring)"""
    job = LocalJob([sys.executable, os.path.join(ROOT, "tests", "scripts", "host_half.py")] +
                   extra, 3, 1, capture=True, timeout=120, print_fn=lambda m: None)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-3000:]
    assert out.count("H16 OK") == 3, out[-3000:]


@pytest.mark.parametrize("lib", ["standard", "base", "mock", "empty"])
def test_libraries_match_sources(native_build, lib):
    """every in-tree library carries the sha256 of the csrc/ sources it was built from (the
    Makefile compiles it into RabitBuildInfo) and gfx950 device code: a library older than its
    sources fails here instead of silently testing stale code"""
    from rabit_amd import _lib

    info = _lib.build_info(lib)
    assert info["offload_arch"] == "gfx950", info
    assert info["fresh"], ("rebuild with `make -j8`: %s was built from sources with sha256 %s, "
                           "the tree has %s" % (info["library"], info["src_sha256"],
                                                _lib.source_hash()))

