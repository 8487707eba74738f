"""Host wake-up after a synchronisation: a tiny kernel + torch.cuda.synchronize(), timed on the host,
with the HIP runtime's default scheduling or spin-waiting (hipSetDeviceFlags(hipDeviceScheduleSpin)
before the device is first used).  Usage: python tools/sync_probe.py auto|spin|yield|blocking"""
import ctypes
import statistics
import sys
import time

FLAGS = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}
mode = sys.argv[1] if len(sys.argv) > 1 else "auto"
rc = None
if mode != "auto":
    rc = ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(FLAGS[mode])
import torch  # noqa: E402

x = torch.zeros(1, device="cuda")
for _ in range(200):
    x.add_(1)
torch.cuda.synchronize()
ts = []
for _ in range(2000):
    t0 = time.perf_counter()
    x.add_(1)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e6)
print(f"{mode}: hipSetDeviceFlags rc={rc}; launch + synchronize median {statistics.median(ts):.1f} us, "
      f"p10 {sorted(ts)[200]:.1f}, p90 {sorted(ts)[1800]:.1f}")
