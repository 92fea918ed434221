import sys, numpy as np
sys.path.insert(0, "clip-embedder-rs_amd")
from open_clip_inference import _lib
L = _lib.lib()
x = np.arange(64, dtype=np.float32) + 1
out = np.empty(512, np.float32)
_lib.check(L.clipgpu_test_lane_reduce(x.ctypes.data, out.ctypes.data))
o = out.reshape(8, 64)
np.set_printoptions(linewidth=250)
for k, name in enumerate(["wave_sum", "wave_max", "xsum16", "xsum32", "row16sum", "row16max", "r16_0", "r16_1"]):
    print(name, o[k].astype(int))
