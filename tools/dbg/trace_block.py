"""Debug: run one saved block through a -DLZ4E_TRACE build (LZ4E_LIB) and
save the event trace to gpurun_out/dbg/<name>.trace (u64 pairs)."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa

name, cls = sys.argv[1], int(sys.argv[2])
data = open(os.path.join(REPO, "exp", name + ".in"), "rb").read()
L = lz4e_amd.lib()
P = ctypes.c_void_p
L.lz4e_debug_compress_stamped.argtypes = [P] * 8 + [ctypes.c_uint32, ctypes.c_uint32, P, P]
dev = torch.device("cuda")
src = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).to(dev)
n = len(data)
cap = n + n // 255 + 16
dst = torch.zeros(cap + 64, dtype=torch.uint8, device=dev)
t = lambda a, dt: torch.tensor(a, dtype=dt, device=dev)
offs, lens, tt, doffs, caps = t([0], torch.int64), t([n], torch.int32), t([cls], torch.uint8), t([0], torch.int64), t([cap], torch.int32)
ret = t([-7], torch.int32)
dbg = torch.zeros(8 + 2 * (1 << 16), dtype=torch.int64, device=dev)
rc = L.lz4e_debug_compress_stamped(src.data_ptr(), offs.data_ptr(), lens.data_ptr(), tt.data_ptr(), dst.data_ptr(),
                                   doffs.data_ptr(), caps.data_ptr(), ret.data_ptr(), 1, n, None, dbg.data_ptr())
torch.cuda.synchronize()
print("rc", rc, "ret", int(ret[0]))
dbg.cpu().numpy()[8:].tofile(os.path.join(REPO, "gpurun_out", "dbg", name + ".trace"))
frame = dst[: int(ret[0])].cpu().numpy().tobytes()
open(os.path.join(REPO, "gpurun_out", "dbg", name + ".tracegpu"), "wb").write(frame)
