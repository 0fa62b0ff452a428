"""Per-kernel timeline of one learner step from in-kernel s_memrealtime stamps.

usage (GPU box): [ALGO=dqn|double|per|mgsc] python tools/trace_step.py
(builds libdqz_trace.so first, unless DQZ_TRACE_PREBUILT=1)
Prints, per kernel in launch order: first-block start relative to the previous
kernel's last-block end (the boundary), kernel span, median block lifetime and
the median of the named intervals between stamps (10 ns ticks -> us).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get('DQZ_TRACE_LIB') or os.path.join(ROOT, 'dqn_mgsc_zoo_amd', 'libdqz_trace.so')  # prebuilt variants
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402
if os.environ.get('DQZ_TRACE_PREBUILT') != '1':  # 1: libdqz_trace.so was built beforehand (off the GPU box)
  __graft_entry__._compile_lib(LIB, ['-DDQZ_TRACE', *os.environ.get('DQZ_TRACE_FLAGS', '').split()])  # pylint: disable=protected-access
os.environ['DQZ_LIB'] = LIB
from dqn_mgsc_zoo_amd import _native as _nat  # noqa: E402
_nat.LIB_PATH = LIB  # imported by the build above, before DQZ_LIB was set
import torch  # noqa: E402
from dqn_mgsc_zoo_amd import _native, learner as learner_lib, networks, synthetic  # noqa: E402

NAMES = {10: 'sample', 0: 'conv1_fwd', 1: 'conv2_fwd', 2: 'conv3_fwd', 3: 'fc1_fwd', 4: 'head', 5: 'fc1_dx',
         6: 'conv3_dx', 7: 'conv2_dx', 8: 'conv1_dw', 9: 'update', 11: 'fc1_dw*', 12: 'conv3_dw*', 13: 'conv2_dw*', 14: 'c1_stage*', 15: 'head_sub*'}
ORDER = [10, 0, 14, 1, 2, 3, 4, 15, 5, 6, 11, 7, 12, 8, 13, 9]
K, NB, NS = 20, 4096, 4  # common.hpp TRACE_*: kernels 16-18 are the HVP launches (tools/trace_hvp.py)

dev = torch.device('cuda:0')
cap = int(os.environ.get('CAP', '200000'))
ALGO = os.environ.get('ALGO', 'dqn')  # dqn | double | per | mgsc: bench.py's workloads
BATCH = int(os.environ.get('BATCH', '32'))  # dqn: BATCH=1 is the MGSC theta' pass's shape
if ALGO == 'dqn':
  net = networks.dqn_atari_network(6)
  lrn = learner_lib.Learner(net, BATCH, algo='dqn', device=dev)
  lrn.set_params(net.init(0))
  store = synthetic.fill_episodic(cap, 6, seed=0, device=dev)
  slots = torch.zeros((BATCH,), dtype=torch.int32, device=dev)
  counter = torch.zeros((1,), dtype=torch.int64, device=dev)

  def step():
    lrn.step_uniform(store, 0, cap, cap, 1, counter, slots)
else:
  import bench  # noqa: E402  (its workloads: the PER / learned-logit draws inside the step)
  wl = bench.Workload(ALGO, cap, 0, dev)
  step = wl.one_step


lib = _native.lib()
fn = lib.dqz_debug_trace
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(K * NB * NS, np.uint64)
side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
  for _ in range(3):
    step()
torch.cuda.current_stream(dev).wait_stream(side)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
  for _ in range(20):
    step()
for _ in range(5):
  g.replay()
torch.cuda.synchronize()
fn(None, 1)
g.replay()
torch.cuda.synchronize()
fn(buf.ctypes.data, 0)
t = buf.reshape(K, NB, NS).astype(np.int64)
prev_end = None
t0 = t[:, :, 0][t[:, :, 0] > 0].min()
print('%-10s %8s %8s %8s | %8s %8s %8s %8s  (us; 100 MHz ticks)' % (
    'kernel', 'gap', 'span', 'blk_med', 's0-s1', 's1-s2', 's2-s3', 'nblk'))
for k in ORDER:
  if k == 14:  # conv1 fwd staging sub-stamps: start -> slot, slot -> frame loads issued, -> LDS staged
    ok = (t[14, :, 0] > 0) & (t[0, :, 0] > 0)
    if ok.any():
      d = lambda a, b: np.median(a[ok] - b[ok]) / 100
      print('%-10s start->slot %.2f  slot->fidx+issue %.2f  ->frames staged %.2f  ->W staged %.2f' % (
          'c1_stage', d(t[14, :, 0], t[0, :, 0]), d(t[14, :, 1], t[14, :, 0]), d(t[14, :, 2], t[14, :, 1]),
          d(t[0, :, 1], t[14, :, 2])))
    continue
  if k == 15:  # head sub-stamps: start -> h(z=0) -> wave sums -> q in LDS -> dz1 stored
    ok = (t[15, :, 0] > 0) & (t[4, :, 0] > 0)
    if ok.any():
      d = lambda a, b: np.median(a[ok] - b[ok]) / 100
      print('%-10s start->h %.2f  ->wave sums %.2f  ->q %.2f  ->TD+dz1 %.2f' % (
          'head_sub', d(t[15, :, 0], t[4, :, 0]), d(t[15, :, 1], t[15, :, 0]), d(t[15, :, 2], t[15, :, 1]),
          d(t[4, :, 3], t[15, :, 2])))
    continue
  s0 = t[k, :, 0]
  live = s0 > 0
  if not live.any():
    continue
  s0 = s0[live]
  s3 = t[k, live, 3]
  start, end = s0.min(), s3.max()
  gap = (start - prev_end) / 100 if prev_end is not None else 0
  def med(a, b):
    x = t[k, live, b] - t[k, live, a]
    ok = (t[k, live, a] > 0) & (t[k, live, b] > 0)
    return np.median(x[ok]) / 100 if ok.any() else float('nan')
  print('%-10s %8.2f %8.2f %8.2f | %8.2f %8.2f %8.2f %8d  [%.2f .. %.2f]' % (
      NAMES[k], gap, (end - start) / 100, np.median(s3 - s0) / 100, med(0, 1), med(1, 2), med(2, 3), live.sum(),
      (start - t0) / 100, (end - t0) / 100))
  if os.environ.get('PCT'):  # start / end percentiles 0, 10, 50, 90, 100
    q = lambda a: ' '.join('%.2f' % ((np.percentile(a, p) - t0) / 100) for p in (0, 10, 50, 90, 100))
    print('%10s start %s | end %s' % ('', q(s0), q(s3)))
  rng = os.environ.get('RANGES_%d' % k)  # e.g. RANGES_9=0,257,1283,2437: per-block-range end percentiles
  if rng:
    cuts = [int(x) for x in rng.split(',')] + [NB]
    for lo, hi in zip(cuts[:-1], cuts[1:]):
      sel = t[k, lo:hi, 0] > 0
      if sel.any():
        e = t[k, lo:hi, 3][sel]
        b0 = t[k, lo:hi, 0][sel]
        print('%10s blocks [%d, %d): start p50 %.2f | end p50 %.2f p90 %.2f max %.2f | life p50 %.2f' % (
            '', lo, hi, (np.median(b0) - t0) / 100, (np.median(e) - t0) / 100,
            (np.percentile(e, 90) - t0) / 100, (e.max() - t0) / 100, np.median(e - b0) / 100))
  if not NAMES[k].endswith('*'):
    prev_end = end
