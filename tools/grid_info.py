"""Persistent-grid blocks per CU of each kernel variant (dev tool, under gpurun)."""
import sys

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
lib = rtamd.hip_lib()
print({v: lib.rt_debug_blocks_per_cu(gpu._h, v) for v in range(4)}, flush=True)
