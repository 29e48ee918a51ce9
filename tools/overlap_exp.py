"""Experiment: does overlapping decode with compress shorten the step?

 serial   -- the bench step: compress the batch, then decode it (one stream);
 split    -- within one step: the light blocks (compress ratio < 1.25 in a
             first pass) compressed and decoded on a second stream while the
             heavy blocks compress on the first, then the heavy blocks decode;
 pipeline -- across steps: step k's decode (stream B) overlaps step k+1's
             compress (stream A), two frame buffers alternating.
Every mode's frames and outputs are checked after its timed run.
Usage: python tools/overlap_exp.py [workload] [steps]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    import torch
    import lz4e_amd
    w = sys.argv[1] if len(sys.argv) > 1 else "silesia64k"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    assert lz4e_amd.gpu_available(), lz4e_amd.last_error()
    bs, cls, gen, seg, desc = bench.WORKLOADS[w]
    nblk = bench.DEFAULT_BLOCKS[w]
    U = min(nblk * bs, bench.TOTAL_BYTES.get(w, nblk * bs))
    lens = np.full(nblk, bs, dtype=np.int64)
    lens[-1] = U - (nblk - 1) * bs
    host = np.zeros(nblk * bs, np.uint8)
    host[:U] = bench.make_data(gen, U, bench.CORPUS_SEED)
    d_src = torch.from_numpy(host).to(dev)
    A = bench.Batch(d_src, lens, bs, cls, dev)
    B = bench.Batch(d_src, lens, bs, cls, dev)
    sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    class Sub:
        """Persistent descriptor tensors of a block subset (a kernel on a
        side stream must not read temporaries the allocator may recycle)."""

        def __init__(self, b, idx):
            self.idx = idx
            g = lambda t: t.index_select(0, idx).contiguous()
            self.off, self.len, self.tt = g(b.d_off), g(b.d_len), g(b.d_tt)
            self.doff, self.cap = g(b.d_doff), g(b.d_cap)
            self.ret = torch.zeros(idx.numel(), dtype=torch.int32, device=dev)
            self.dret = torch.zeros(idx.numel(), dtype=torch.int32, device=dev)

    def comp(b, s, sub=None):
        if sub is not None and sub.idx.numel() == 0:
            return
        off, ln, tt, doff, cap, ret = (b.d_off, b.d_len, b.d_tt, b.d_doff, b.d_cap, b.d_ret) if sub is None \
            else (sub.off, sub.len, sub.tt, sub.doff, sub.cap, sub.ret)
        lz4e_amd.compress_batch_dev(b.d_src, off, ln, tt, b.d_dst, doff, cap, ret, max_len=b.bs,
                                    stream=s.cuda_stream)

    def dec(b, s, sub=None):
        if sub is not None and sub.idx.numel() == 0:
            return
        off, ln, doff, ret, dret = (b.d_off, b.d_len, b.d_doff, b.d_ret, b.d_dret) if sub is None \
            else (sub.off, sub.len, sub.doff, sub.ret, sub.dret)
        lz4e_amd.decompress_batch_dev(b.d_dst, doff, ret, b.d_out, off, ln, dret, stream=s.cuda_stream,
                                      max_cap=b.max_cap)

    # reference frames / light-heavy split from one serial pass
    comp(A, sA)
    dec(A, sA)
    torch.cuda.synchronize()
    ref_ret = A.d_ret.clone()
    ref_frames = A.d_dst.clone()
    ratio = lens / np.maximum(1, ref_ret.cpu().numpy())
    li = np.nonzero(ratio < 1.25)[0]
    hi = np.nonzero(ratio >= 1.25)[0]
    light = Sub(A, torch.from_numpy(li).to(dev))
    heavy = Sub(A, torch.from_numpy(hi).to(dev))
    torch.cuda.synchronize()
    assert light.off.numel() + heavy.off.numel() == nblk
    assert int(light.off.max().item() if li.size else 0) <= (nblk - 1) * bs

    def merge_subs():
        # the split mode's results back into A's full-batch tensors
        for sub in (light, heavy):
            if sub.idx.numel():
                A.d_ret.index_copy_(0, sub.idx, sub.ret)
                A.d_dret.index_copy_(0, sub.idx, sub.dret)

    def check(b, name):
        torch.cuda.synchronize()
        ok = torch.equal(b.d_ret, ref_ret) and torch.equal(b.d_out[:U], d_src[:U]) and \
            bool((b.d_dret.cpu().numpy() == lens).all())
        rets = ref_ret.cpu().numpy()
        for i in range(0, nblk, max(1, nblk // 64)):
            o = int(b.doffs[i])
            ok = ok and torch.equal(b.d_dst[o:o + int(rets[i])], ref_frames[o:o + int(rets[i])])
        b.d_out.zero_()
        b.d_dret.zero_()
        return ok

    def serial(k):
        comp(A, sA)
        dec(A, sA)

    ev_c = [torch.cuda.Event() for _ in range(2)]
    ev_d = [torch.cuda.Event() for _ in range(2)]
    ev_l = torch.cuda.Event()

    def split(k):
        ev_l.record(sA)
        sB.wait_event(ev_l)
        comp(A, sB, light)
        comp(A, sA, heavy)
        dec(A, sB, light)
        dec(A, sA, heavy)
        ev_l.record(sB)
        sA.wait_event(ev_l)

    started = [False, False]

    def pipeline(k):
        b = (A, B)[k & 1]
        if started[k & 1]:
            sA.wait_event(ev_d[k & 1])  # that set's previous decode is done
        comp(b, sA)
        ev_c[k & 1].record(sA)
        sB.wait_event(ev_c[k & 1])
        dec(b, sB)
        ev_d[k & 1].record(sB)
        started[k & 1] = True

    res = {"workload": w, "blocks": nblk, "light": int(li.size), "heavy": int(hi.size)}
    for name, f in (("serial", serial), ("split", split), ("pipeline", pipeline), ("serial_again", serial)):
        for k in range(3):
            f(k)
        torch.cuda.synchronize()
        for b in (A, B):
            b.d_out.zero_()
            b.d_dret.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            f(k)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        if name == "split":
            merge_subs()
        ok = check(A, name) and (name != "pipeline" or check(B, name))
        res[name] = {"ms_per_step": round(ms, 4), "GiBps": round(U / ms / 1e-3 / 2**30, 3), "exact": ok}
        started[0] = started[1] = False
    print(res, flush=True)


if __name__ == "__main__":
    main()
