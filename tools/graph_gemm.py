"""Does a captured GEMM replay exactly?  Capture C = A @ B (and A^T/B^T forms) in a hipGraph,
replay it several times and compare every replay with the eager product."""
import json

import torch


def check(m, n, k, ta, tb, lib):
    torch.backends.cuda.preferred_blas_library(lib)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn((k, m) if ta else (m, k), device=dev, generator=g)
    b = torch.randn((n, k) if tb else (k, n), device=dev, generator=g)
    A = a.t() if ta else a
    B = b.t() if tb else b
    ref = A @ B
    c = torch.empty(m, n, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            torch.mm(A, B, out=c)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        torch.mm(A, B, out=c)
    errs = []
    for _ in range(4):
        c.fill_(7.0)
        gr.replay()
        torch.cuda.synchronize()
        errs.append(float((c - ref).abs().max()))
    return {"m": m, "n": n, "k": k, "ta": ta, "tb": tb, "lib": lib, "replay_maxerr": errs}


for lib in ["default", "cublas"]:
    for (m, n, k) in [(1024, 2048, 2048), (2048, 2048, 1024), (1024, 1024, 2000), (512, 1024, 1024),
                      (256, 512, 512)]:
        for ta, tb in [(False, True), (True, False), (False, False)]:
            print(json.dumps(check(m, n, k, ta, tb, lib)), flush=True)
