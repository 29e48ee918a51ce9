"""Diagnostic: per-phase cycles of the one-wave decompress kernel (stamped build).

usage: python tools/dstamps.py [silesia64k,text64k,fio4k,text256k,text256k_16]"""
import ctypes, os, sys
import numpy as np

CLASS_NAMES = ["text", "ints", "runs", "random", "jpeg", "records"]

def by_class(name, tot, n, extra=None):
    if not name.startswith("silesia"):
        return
    cls = np.random.default_rng(0x5157).choice(6, size=n, p=[0.40, 0.15, 0.10, 0.10, 0.10, 0.15])
    for c in range(6):
        m = cls == c
        if m.any():
            print(f"   class {CLASS_NAMES[c]:8s} n={m.sum():4d} mean {tot[m].mean():12.0f} max {tot[m].max():12.0f}" + (f" {extra(m)}" if extra else ""))
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa
from lz4e_amd import corpus  # noqa
L = lz4e_amd.lib()
P = ctypes.c_void_p
L.lz4e_debug_decompress_stamped.argtypes = [P] * 7 + [ctypes.c_uint32, P, P, ctypes.c_uint32, ctypes.c_uint32]

def run(name, data, bs, cls):
    dev = torch.device("cuda")
    n = data.size // bs
    offs = torch.arange(n, dtype=torch.int64, device=dev) * bs
    lens = torch.full((n,), bs, dtype=torch.int32, device=dev)
    tt = torch.full((n,), cls, dtype=torch.uint8, device=dev)
    cap = bs + bs // 255 + 16
    slot = (cap + 79) // 16 * 16
    doffs = torch.arange(n, dtype=torch.int64, device=dev) * slot
    caps = torch.full((n,), cap, dtype=torch.int32, device=dev)
    src = torch.from_numpy(data).to(dev)
    dst = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    ret = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret)
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    dret = torch.zeros(n, dtype=torch.int32, device=dev)
    dbg = torch.zeros(n * 8, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        assert L.lz4e_debug_decompress_stamped(dst.data_ptr(), doffs.data_ptr(), ret.data_ptr(), out.data_ptr(),
                                               offs.data_ptr(), lens.data_ptr(), dret.data_ptr(), n, s,
                                               dbg.data_ptr(), 0, 1) == 0
    torch.cuda.synchronize()
    assert torch.equal(out[:n * bs], src)
    d = dbg.cpu().numpy().reshape(n, 8).astype(np.float64)
    tot = d[:, :3].sum(1) + d[:, 5]
    print(f"== {name}: {n} blocks, cycles/block mean {tot.mean():.0f} max {tot.max():.0f}; batches {d[:,3].mean():.0f} "
          f"rounds {d[:,4].mean():.0f} ({d[:,4].sum()/max(1,d[:,3].sum()):.2f}/batch); parse {d[:,0].mean():.0f} "
          f"lit {d[:,1].mean():.0f} match {d[:,2].mean():.0f} flush {d[:,5].mean():.0f}; cycles/batch {tot.sum()/max(1,d[:,3].sum()):.0f}")
    by_class(name, tot, n, lambda m: f"batches {d[m,3].mean():.0f} rounds {d[m,4].mean():.0f} parse {d[m,0].mean():.0f} lit {d[m,1].mean():.0f} match {d[m,2].mean():.0f}")

W = {"silesia64k": lambda: (corpus.silesia_proxy(1024 * 65536, 0x5157), 65536, 1),
     "text64k": lambda: (corpus.text_proxy(512 * 65536, 7), 65536, 1),
     "fio4k": lambda: (corpus.fio_pattern(16384 * 4096), 4096, 1),
     # configs[4]'s decompress-only leg (one wave per block), full chip and 16 blocks
     "text256k": lambda: (corpus.text_proxy(3815 * 262144, 7), 262144, 3),
     "text256k_16": lambda: (corpus.text_proxy(16 * 262144, 7), 262144, 3)}
for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["silesia64k", "text64k", "fio4k"]):
    run(name, *W[name]())
