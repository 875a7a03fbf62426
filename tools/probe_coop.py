"""Probe (not product code): does hipLaunchCooperativeKernel work eagerly, inside torch's stream
capture and from the replayed graph?  Build: hipcc --offload-arch=gfx950 -shared -fPIC
-o tools/probe_coop.so <the probe source recorded in DESIGN.md>."""
import ctypes
import os
import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe_coop.so"))
lib.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
out = torch.zeros(1, dtype=torch.int32, device="cuda")
grid = 256
s = torch.cuda.current_stream().cuda_stream
print("eager coop rc", lib.probe_launch(cnt.data_ptr(), out.data_ptr(), 1, grid, 1, s), flush=True)
torch.cuda.synchronize()
print("eager result", int(out), "cnt", int(cnt), flush=True)
g = torch.cuda.CUDAGraph()
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    try:
        with torch.cuda.graph(g):
            rc = lib.probe_launch(cnt.data_ptr(), out.data_ptr(), 2, grid, 1, torch.cuda.current_stream().cuda_stream)
        print("capture rc", rc, flush=True)
    except Exception as e:
        print("capture failed:", repr(e)[:300], flush=True)
        raise SystemExit(0)
for ep in (2, 3):
    g.replay()
    torch.cuda.synchronize()
    print("replay", ep, "result", int(out), "cnt", int(cnt), flush=True)

# The probe kernel (tools/probe_coop.so), for the record:
#   extern "C" __global__ void k_probe(unsigned* cnt, unsigned* out, unsigned epoch) {
#       if (threadIdx.x == 0) {
#           __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#           if (blockIdx.x == 0) {              // bounded wait for every block's add
#               unsigned v = 0;
#               for (int it = 0; it < (1 << 22); ++it) {
#                   v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#                   if (v >= epoch * gridDim.x) break;
#                   __builtin_amdgcn_s_sleep(2);
#               }
#               out[0] = v;
#           }
#       }
#   }
#   launched with hipLaunchCooperativeKernel(k_probe, 256 blocks x 64 threads, stream).
# Measured on the MI355X box: eager 256 / 256, captured rc 0, replays 512 and 768: cooperative
# launches capture into and replay from a hipGraph.
