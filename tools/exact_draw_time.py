"""Device time of the learned-logit draws and default-logit adds at 1M slots,
exact mode (dqz_logits_sample_exact / _add_exact) against the default.
usage (GPU box): python tools/exact_draw_time.py"""
import sys, time, numpy as np, torch
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dqn_mgsc_zoo_amd import replay_circular as rc
cap = 1_000_000
rng = np.random.default_rng(0)
dev = rc._DeviceLogits(cap, max_queries=64)
dev.logits.copy_(torch.from_numpy(rng.standard_normal(cap).astype(np.float32)))
u = rng.random(32)
for _ in range(5):
  dev.sample_exact(u); dev.sample_abs(u)
torch.cuda.synchronize()
for name, fn in (('exact draw', lambda: dev.sample_exact(u)), ('default draw', lambda: dev.sample_abs(u)),
                 ('exact add', lambda: dev.add_default_exact(5, cap - 10)),
                 ('default add', lambda: dev.add_default(5, cap - 10))):
  e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
  e0.record()
  for _ in range(200): fn()
  e1.record(); torch.cuda.synchronize()
  print(name, 'us per call (a draw: 32 queries, incl. the H2D copy of u):', round(e0.elapsed_time(e1) / 200 * 1e3, 2))
