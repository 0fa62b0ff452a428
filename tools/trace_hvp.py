"""Timeline of the second-order meta-update's HVP launches (hvp.hpp) from
in-kernel s_memrealtime stamps (DQZ_TRACE builds; kernels 16-18 of the
trace buffer).

usage (GPU box): python tools/trace_hvp.py   (libdqz_trace.so prebuilt by
tools/build_variants.sh, or DQZ_TRACE_LIB=<path>)
Prints per launch and per block range: start / end percentiles relative to
the first stamp of L1, the median block lifetime and the medians of the
stamped intervals (10 ns ticks -> us).  The meta-update runs eagerly three
times, then once more with the stamps cleared before it.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get('DQZ_TRACE_LIB') or os.path.join(ROOT, 'dqn_mgsc_zoo_amd', 'libdqz_trace.so')
os.environ['DQZ_LIB'] = LIB
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from dqn_mgsc_zoo_amd import _native, learner as learner_lib, networks, replay as replay_lib, synthetic  # noqa: E402
from dqn_mgsc_zoo_amd import replay_circular as rc  # noqa: E402

K, NB, NS = 20, 4096, 4  # common.hpp TRACE_*
B, A, M = 32, 6, 100
# block ranges per launch (hvp.hpp): name, first block
RANGES = {
    16: ('L1', [('t12', 0), ('s1', 324), ('b3', 325)], 521, ('tile staged', 'ty1 reduced')),
    17: ('L2', [('t34', 0), ('b2', 196)], 520, ('ty3 sums', '')),
    18: ('L3', [('b1', 0), ('g hidden', 400), ('g conv2', 408), ('g conv3', 921), ('g conv1', 1498),
                ('g fc1', 1755)], 2147, ('x staged', 'ddot1 wait')),
}


def main():
  dev = torch.device('cuda:0')
  cap = 200_000
  store = synthetic.fill_episodic(cap, A, seed=0, device=dev)
  rng = np.random.default_rng(0)
  net = networks.dqn_atari_network(A)
  lrn = learner_lib.Learner(net, B, algo='dqn', device=dev)
  lrn.set_params(net.init(seed=3))
  lbuf = rc._DeviceLogits(cap, dev, max_queries=B)  # pylint: disable=protected-access
  lbuf.load(rng.standard_normal(cap).astype(np.float32))
  lbuf.sample_abs(rng.random(B))
  ot = replay_lib.Transition(rng.integers(0, 256, (84, 84, 4), dtype=np.uint8), 2, 1.0, 0.99,
                             rng.integers(0, 256, (84, 84, 4), dtype=np.uint8))
  meta = learner_lib.MetaLearner(lrn, M, learner_lib.adam(2.5e-4), second_order=True)
  meta.set_online_transition(ot)
  ms = torch.from_numpy(rng.choice(cap, M, replace=False).astype(np.int32)).to(dev)
  fn = _native.lib().dqz_debug_trace_other  # the HVP kernels' code object
  fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
  buf = np.zeros(K * NB * NS, np.uint64)
  for _ in range(3):
    meta.update(store, ms, lbuf.logits, ms, logit_buffer=lbuf)
  torch.cuda.synchronize()
  fn(None, 1)
  meta.update(store, ms, lbuf.logits, ms, logit_buffer=lbuf)
  torch.cuda.synchronize()
  fn(buf.ctypes.data, 0)
  t = buf.reshape(K, NB, NS).astype(np.int64)
  t0 = t[16, :, 0][t[16, :, 0] > 0].min()
  us = lambda x: (x - t0) / 100
  prev_end = None
  for k in (16, 17, 18):
    name, ranges, nblk, labels = RANGES[k]
    live = t[k, :nblk, 0] > 0
    if not live.any():
      print(name, 'no stamps')
      continue
    s0, s3 = t[k, :nblk, 0][live], t[k, :nblk, 3][live]
    gap = (s0.min() - prev_end) / 100 if prev_end is not None else 0.0
    print('%s: gap %.2f  span %.2f  [%.2f .. %.2f]  blocks %d' % (name, gap, (s3.max() - s0.min()) / 100, us(s0.min()),
                                                               us(s3.max()), live.sum()))
    prev_end = s3.max()
    bounds = [r[1] for r in ranges] + [nblk]
    for (rn, lo), hi in zip(ranges, bounds[1:]):
      sel = t[k, lo:hi, 0] > 0
      if not sel.any():
        continue
      b0, b3 = t[k, lo:hi, 0][sel], t[k, lo:hi, 3][sel]
      line = '  %-9s [%4d, %4d) start p0 %.2f p50 %.2f max %.2f | end p50 %.2f p90 %.2f max %.2f | life p50 %.2f' % (
          rn, lo, hi, us(b0.min()), us(np.median(b0)), us(b0.max()), us(np.median(b3)), us(np.percentile(b3, 90)),
          us(b3.max()), np.median(b3 - b0) / 100)
      for j, lab in enumerate(labels):
        s = t[k, lo:hi, j + 1][sel]
        if lab and (s > 0).all():
          prev = t[k, lo:hi, j][sel] if j else b0
          line += ' | ->%s %.2f' % (lab, np.median(s - prev) / 100)
      print(line)


if __name__ == '__main__':
  main()
