#!/usr/bin/env python3
"""Host cost of one kernel launch through the engine library
(crdtm_xbench_launch) in a process that has torch's HIP runtime up: on a
stream of the library's own and on torch's current stream; then the same
inside the engine's own context (crdtm_ctx_create on torch's stream)."""
import ctypes as C
import os

import torch

here = os.path.dirname(os.path.abspath(__file__))
torch.zeros(1, device="cuda")
lib = C.CDLL(os.path.join(here, "..", "crdt-graph_amd", "crdtm", "libcrdtm.so"))
f = lib.crdtm_xbench_launch
f.restype = C.c_double
f.argtypes = [C.c_void_p, C.c_int]
print("torch up, own stream: %.2f us" % f(None, 2000), flush=True)
s = torch.cuda.current_stream()
print("torch current stream: %.2f us" % f(C.c_void_p(s.cuda_stream), 2000), flush=True)
x = torch.zeros(1 << 20, device="cuda")
print("after a torch kernel: %.2f us" % f(C.c_void_p(s.cuda_stream), 2000), flush=True)
