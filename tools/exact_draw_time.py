import sys, time, numpy as np, torch
sys.path.insert(0, '.')
from dqn_mgsc_zoo_amd import replay_circular as rc
cap = 1_000_000
rng = np.random.default_rng(0)
dev = rc._DeviceLogits(cap, max_queries=64)
dev.logits.copy_(torch.from_numpy(rng.standard_normal(cap).astype(np.float32)))
u = rng.random(32)
for _ in range(5):
  dev.sample_exact(u); dev.sample_abs(u)
torch.cuda.synchronize()
for name, fn in (('exact', lambda: dev.sample_exact(u)), ('fast', lambda: dev.sample_abs(u))):
  e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
  e0.record()
  for _ in range(200): fn()
  e1.record(); torch.cuda.synchronize()
  print(name, 'us per 32-draw call (incl. H2D of u):', round(e0.elapsed_time(e1) / 200 * 1e3, 2))
