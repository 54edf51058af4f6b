"""kepler_amd — MI355X-native engine for Kepler's power-attribution hot path.

Package layout:
  csrc/      HIP kernels for gfx950 + the C ABI (include/kepler_accel.h)
  lib/       in-tree build output (libkepler_accel.so)
  accel.py   ctypes binding of the C ABI (the Python twin of the cgo shim)
  fleet.py   synthetic fleet generator / SoA batch layout
  monitor.py host-side mirror of monitor.PowerMonitor over the engine
"""

__all__ = ["accel", "fleet"]
