"""Fused round trip (tools/rtexp/librt.so: one launch compresses each block
and decodes its own frame) against the two-launch step of bench.py, on the
bench workloads.  Checks the fused frames and outputs equal the product's.

Usage: python tools/rtexp/rtbench.py [workloads] [steps]
"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import bench  # noqa: E402


def main():
    import torch
    import lz4e_amd
    works = (sys.argv[1] if len(sys.argv) > 1 else "silesia64k,text256k,fio4k,sg512").split(",")
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rt = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt.so"))
    rt.rt_roundtrip_dev.restype = ctypes.c_int
    rt.rt_roundtrip_dev.argtypes = [ctypes.c_void_p] * 11 + [ctypes.c_uint32, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    assert lz4e_amd.gpu_available(), lz4e_amd.last_error()
    for w in works:
        bs, cls, gen, seg, desc = bench.WORKLOADS[w]
        nblk = bench.DEFAULT_BLOCKS[w]
        U = min(nblk * bs, bench.TOTAL_BYTES.get(w, nblk * bs))
        lens = np.full(nblk, bs, dtype=np.int64)
        lens[-1] = U - (nblk - 1) * bs
        host = np.zeros(nblk * bs, np.uint8)
        host[:U] = bench.make_data(gen, U, bench.CORPUS_SEED)
        b = bench.Batch(torch.from_numpy(host).to(dev), lens, bs, cls, dev)
        f_dst = torch.zeros_like(b.d_dst)
        f_ret = torch.zeros_like(b.d_ret)
        f_out = torch.zeros_like(b.d_out)
        f_dret = torch.zeros_like(b.d_dret)
        s = b.stream.cuda_stream

        def fused():
            r = rt.rt_roundtrip_dev(b.d_src.data_ptr(), b.d_off.data_ptr(), b.d_len.data_ptr(),
                                    b.d_tt.data_ptr(), f_dst.data_ptr(), b.d_doff.data_ptr(),
                                    f_ret.data_ptr(), f_out.data_ptr(), b.d_off.data_ptr(),
                                    b.d_len.data_ptr(), f_dret.data_ptr(), nblk, s)
            assert r == 0

        def two():
            b.compress()
            b.decompress()

        for f in (two, fused):
            f()
        torch.cuda.synchronize()
        same = (torch.equal(f_ret, b.d_ret) and torch.equal(f_dret, b.d_dret)
                and torch.equal(f_out[:U], b.d_src[:U]) and torch.equal(b.d_out[:U], b.d_src[:U]))
        rets = b.d_ret.cpu().numpy()
        for i in range(nblk):
            o, n = int(b.doffs[i]), int(rets[i])
            if not torch.equal(f_dst[o:o + n], b.d_dst[o:o + n]):
                same = False
                break
        res = {}
        for name, f in (("two_launch", two), ("fused", fused), ("two_launch_again", two)):
            for _ in range(3):
                f()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev[0].record(b.stream)
            for _ in range(steps):
                f()
            ev[1].record(b.stream)
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / steps
            res[name] = {"ms_per_step": round(ms, 4), "GiBps": round(U / ms / 1e-3 / 2**30, 3),
                         "wall_ms": round((time.perf_counter() - t0) * 1e3 / steps, 4)}
        print({"workload": w, "blocks": nblk, "identical": same, **res}, flush=True)


if __name__ == "__main__":
    main()
