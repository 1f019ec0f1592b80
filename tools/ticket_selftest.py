"""Diagnosis: the ticket protocol with trivial items (mpiv_selftest_tickets, libmpiv_ab.so)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_vision_amd import _lib  # noqa: E402

blocks, nphase, nvirt = (int(a) for a in sys.argv[1:4])
dev = torch.device("cuda:0")
L = _lib.load_ab()
ctr = torch.zeros(4, dtype=torch.int32, device=dev)
marks = torch.zeros(nphase * nvirt, dtype=torch.int32, device=dev)
print("launch", blocks, nphase, nvirt, flush=True)
rc = L.mpiv_selftest_tickets(blocks, nphase, nvirt, 1 << 22, ctypes.c_void_p(ctr.data_ptr()),
                             ctypes.c_void_p(marks.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
assert rc == 0, L.mpiv_last_error()
torch.cuda.synchronize()
print("ctr", ctr.tolist(), "marks", int(marks.sum().item()), "of", nphase * nvirt, flush=True)
