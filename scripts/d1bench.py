import os, sys, time
import numpy as np
sys.path.insert(0, "3dy4-real-time-software-defined-radio-_amd")
import sdrhip
ctx = sdrhip.Context(0)
S, n = 1024, 5120
rng = np.random.default_rng(1)
x = rng.standard_normal((S, n)).astype(np.float32)
h = (rng.standard_normal(101) / 101).astype(np.float32)
A = sdrhip.DeviceArray
d_x = A.from_numpy(ctx, x); d_h = A.from_numpy(ctx, h); d_st = A.from_numpy(ctx, np.zeros(S * 100, np.float32)); d_y = A(ctx, S * n * 4)
for _ in range(3): ctx.fir_block_dev(d_x, n, S, n, d_h, 101, d_st, 100, d_y, n)
ctx.synchronize(); t0 = time.perf_counter()
for _ in range(50): ctx.fir_block_dev(d_x, n, S, n, d_h, 101, d_st, 100, d_y, n)
ctx.synchronize(); print(os.environ.get("SDRHIP_LIB","").split("/")[-1], "D=1 FIR 1024x5120:", (time.perf_counter() - t0) / 50 * 1e6, "us")
