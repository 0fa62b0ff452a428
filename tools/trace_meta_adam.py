"""Timeline of meta_adam_chunks_kernel (meta.hpp) from in-kernel
s_memrealtime stamps (DQZ_TRACE builds; kernel 19 of the trace buffer).

usage (GPU box): python tools/trace_meta_adam.py [capacity]   (libdqz_trace.so
prebuilt by tools/build_variants.sh, or DQZ_TRACE_LIB=<path>)
Stamps: 0 entry (every block), 1 entry loads returned (active blocks),
2 before the dS reduction (after the leader's wait), 3 end of the common
path.  Prints, relative to the first entry stamp (10 ns ticks -> us), the
spread of the entry stamps over all blocks, the active blocks' intervals and
the leader's.  A first-order meta-update runs eagerly three times, then once
more with the stamps cleared before it.
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
KID = 19
B, A, M = 32, 6, 100
CHUNK = 4096  # sampling.hpp SM_CHUNK


def pct(x):
  return 'p0 %6.2f p50 %6.2f p90 %6.2f max %6.2f' % (x.min(), np.median(x), np.percentile(x, 90), x.max())


def main():
  cap = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
  dev = torch.device('cuda:0')
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
  meta = learner_lib.MetaLearner(lrn, M, learner_lib.adam(2.5e-4), second_order=False)
  meta.set_online_transition(ot)
  pos = rng.choice(cap, M, replace=False).astype(np.int32)
  ms = torch.from_numpy(pos).to(dev)
  fn = _native.lib().dqz_debug_trace_other
  fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
  buf = np.zeros(K * NB * NS, np.uint64)
  for _ in range(3):
    meta.update(store, ms, lbuf.logits, ms, logit_buffer=lbuf)
  torch.cuda.synchronize()
  fn(None, 1)
  meta.update(store, ms, lbuf.logits, ms, logit_buffer=lbuf)
  torch.cuda.synchronize()
  fn(buf.ctypes.data, 0)
  full = buf.reshape(K, NB, NS).astype(np.int64)
  nblk = (cap + CHUNK - 1) // CHUNK
  t = full[KID, :nblk]
  # finer stamps (kernels 13 / 12 of this code object's buffer): s row summed, tot reduced, Adam arithmetic
  # done | dS reduced; lane chunk terms done, chunk scan done
  t13, t12 = full[13, :nblk], full[12, :nblk]
  live = t[:, 0] > 0
  t0 = t[live, 0].min()
  us = lambda x: (x - t0) / 100
  act = np.zeros(nblk, bool)
  act[np.unique(pos // CHUNK)] = True
  leader = pos[0] // CHUNK
  print('capacity %d blocks %d stamped %d active %d leader %d' % (cap, nblk, live.sum(), act.sum(), leader))
  print('entry, all blocks      ', pct(us(t[live, 0])))
  print('entry, active blocks   ', pct(us(t[act, 0])))
  a = t[act]
  ok = (a[:, 1:] > 0).all(axis=1)
  a = a[ok]
  print('loads back (1)         ', pct(us(a[:, 1])), '| 1-0 p50 %.2f' % (np.median(a[:, 1] - a[:, 0]) / 100))
  print('before dS (2)          ', pct(us(a[:, 2])), '| 2-1 p50 %.2f' % (np.median(a[:, 2] - a[:, 1]) / 100))
  print('end (3)                ', pct(us(a[:, 3])), '| 3-2 p50 %.2f' % (np.median(a[:, 3] - a[:, 2]) / 100))
  a13, a12 = t13[act][ok], t12[act][ok]
  if (a13 > 0).all() and (a12[:, :2] > 0).all():
    seq = [('loads back', a[:, 1]), ('s row', a13[:, 0]), ('tot', a13[:, 1]), ('adam', a13[:, 2]),
           ('before dS', a[:, 2]), ('dS', a13[:, 3]), ('lane terms', a12[:, 0]), ('chunk scan', a12[:, 1]),
           ('end', a[:, 3])]
    print('active-block intervals (p50 us):', ' '.join(
        '%s->%s %.2f' % (p[0], q[0], np.median(q[1] - p[1]) / 100) for p, q in zip(seq, seq[1:])))
  lt = t[leader]
  print('leader: entry %.2f loads %.2f after wait %.2f end %.2f' % tuple(us(lt[j]) for j in range(4)))
  inact = live & ~act
  if inact.any():
    print('inactive blocks: entry', pct(us(t[inact, 0])))


if __name__ == '__main__':
  main()
