"""us per MGSC replay add at the reference's 1M capacity (GPU box).

FIFO CircularLogitBuffer full at 1M: popleft + default add (log-mean-exp of
all logits), the reference's 1.94 ms/add path.  Device time
per add from HIP events over 2000 adds, for the running log-sum-exp and for a
full re-scan per add (invalidate before each add).  Prints one JSON line.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dqn_mgsc_zoo_amd import replay_circular as rc  # noqa: E402

cap = 1_000_000
buf = rc.CircularLogitBuffer(cap, np.random.default_rng(0))
dev = buf._dev  # pylint: disable=protected-access
dev.load(np.random.default_rng(1).standard_normal(cap).astype(np.float32))
buf._size = cap  # pylint: disable=protected-access
out = {}
for mode in ('running', 'rescan'):
  for _ in range(50):
    buf.popleft(return_value=False)
    buf.add()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  n = 2000
  t = time.perf_counter()
  e0.record()
  for _ in range(n):
    if mode == 'rescan':
      dev.invalidate()
    buf.popleft(return_value=False)
    buf.add()
  e1.record()
  torch.cuda.synchronize()
  out[mode] = {'device_us_per_add': round(e0.elapsed_time(e1) * 1e3 / n, 2),
               'host_us_per_add': round((time.perf_counter() - t) * 1e6 / n, 2)}
out['reference_ms_per_add'] = 1.94
print(json.dumps(out))
