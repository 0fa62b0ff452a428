"""Generates tests/golden/replay_golden.json from the REFERENCE replay code.

Runs only in the build container, where /root/reference exists (it is never
needed on the GPU box: the JSON output is committed).  The reference modules
`dqn_zoo/replay.py` and `dqn_zoo/replay_circular.py` import jax, snappy,
dm_env and dqn_zoo.parts at top level but do not use them on the numpy code
paths exercised here, so those names are stubbed in sys.modules.  Nothing
from the reference is copied: this script only records inputs and the
reference's outputs.

numpy %s at generation time (Generator / RandomState streams are
version-stable for the calls used: randint, integers, uniform, choice).
"""

import importlib
import json
import os
import sys
import types

import numpy as np

REF = '/root/reference'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                   'replay_golden.json')


def _load_reference():
  jax = types.ModuleType('jax')
  jnp = types.ModuleType('jax.numpy')
  jnp.ndarray = np.ndarray
  jax.numpy = jnp
  sys.modules.setdefault('jax', jax)
  sys.modules.setdefault('jax.numpy', jnp)
  sys.modules.setdefault('snappy', types.ModuleType('snappy'))
  dm = types.ModuleType('dm_env')
  dm.TimeStep = object
  dm.StepType = object
  sys.modules.setdefault('dm_env', dm)
  pkg = types.ModuleType('dqn_zoo')
  pkg.__path__ = [os.path.join(REF, 'dqn_zoo')]
  sys.modules['dqn_zoo'] = pkg
  parts = types.ModuleType('dqn_zoo.parts')
  parts.Action = int
  sys.modules['dqn_zoo.parts'] = parts
  pkg.parts = parts
  return (importlib.import_module('dqn_zoo.replay'),
          importlib.import_module('dqn_zoo.replay_circular'))


def _f(x):
  return np.asarray(x, np.float64).tolist()


def _i(x):
  return np.asarray(x, np.int64).tolist()


def sumtree_cases(replay):
  out = {}
  # known-answer table of replay_test.py (values [3,1,2,5])
  t = replay.SumTree()
  t.set_all([3.0, 1.0, 2.0, 5.0])
  targets = [0.0, 2.9, 3.0, 3.9, 4.0, 5.9, 6.0, 10.9, 2.9, 4.0]
  out['query_table'] = {'values': [3.0, 1.0, 2.0, 5.0], 'targets': targets,
                        'indices': _i(t.query(targets))}
  # random operation streams (resize / set / set_all / query)
  streams = []
  for seed in range(6):
    rs = np.random.RandomState(seed)
    t = replay.SumTree()
    ops = []
    for _ in range(12):
      n = int(rs.randint(10, 40))
      t.resize(n)
      ops.append(['resize', n])
      idx = rs.randint(t.size, size=3)
      vals = np.abs(rs.standard_cauchy(3))
      t.set(idx, vals)
      ops.append(['set', _i(idx), _f(vals)])
      tg = rs.uniform(0, t.root(), size=4)
      ops.append(['query', _f(tg), _i(t.query(tg)), float(t.root())])
      vals = np.abs(rs.standard_cauchy(int(rs.randint(10, 40))))
      t.set_all(vals)
      ops.append(['set_all', _f(vals)])
      tg = rs.uniform(0, t.root(), size=3)
      ops.append(['query', _f(tg), _i(t.query(tg)), float(t.root())])
    streams.append({'ops': ops, 'final_values': _f(t.values),
                    'capacity': int(t.capacity)})
  out['streams'] = streams
  return out


def uniform_replay_cases(replay):
  cases = []
  for seed, capacity, n_add, sizes in ((1, 10, 31, [3, 5]), (7, 50, 120, [32]),
                                       (3, 5, 5, [2, 4])):
    rs = np.random.RandomState(seed)
    r = replay.TransitionReplay(capacity, replay.Transition(None, None, None, None, None), rs)
    log = []
    for i in range(n_add):
      r.add(replay.Transition(i, i % 4, float(i), 0.99, i + 1))
      if i >= 2 and i % 3 == 0:
        for sz in sizes:
          s = r.sample(sz)
          log.append({'after_add': i, 'size': sz, 'ids': _i(s.s_tm1)})
    cases.append({'seed': seed, 'capacity': capacity, 'n_add': n_add,
                  'sizes': sizes, 'samples': log, 'final_ids': _i(list(r.ids()))})
  return cases


def reservoir_cases(replay, rc):
  out = []
  for mod_name, mod in (('replay', replay), ('replay_circular', rc)):
    for seed in (0, 5):
      rng = (np.random.RandomState(seed) if mod_name == 'replay' else
             np.random.default_rng(seed))
      r = mod.ReservoirTransitionReplay(
          20, mod.Transition(None, None, None, None, None), rng)
      for i in range(100):
        r.add(mod.Transition(i, 0, 0.0, 1.0, i))
      stored = [int(x.s_tm1) for x in r.get(sorted(r.ids()))]
      s = r.sample(16)
      out.append({'module': mod_name, 'seed': seed, 'capacity': 20,
                  'n_add': 100, 'slot_items': stored,
                  'sample_items': _i(s.s_tm1)})
  return out


def prioritized_cases(replay):
  out = []
  for seed in (1, 2):
    rs = np.random.RandomState(seed)
    r = replay.PrioritizedTransitionReplay(
        capacity=8, structure=replay.Transition(None, None, None, None, None),
        priority_exponent=0.6, importance_sampling_exponent=lambda t: 0.4,
        uniform_sample_probability=0.1, normalize_weights=True, random_state=rs)
    prios = [1.0, 0.5, 2.0, 0.0, 3.0, 1.5, 0.25, 4.0, 2.5, 0.75, 1.25]
    log = []
    for i, p in enumerate(prios):
      r.add(replay.Transition(i, 0, 0.0, 1.0, i), priority=p)
      if i >= 3:
        tr, ids, w = r.sample(5)
        log.append({'after_add': i, 'ids': _i(ids), 'items': _i(tr.s_tm1),
                    'weights': _f(w)})
        r.update_priorities(ids[:2], [0.3 * (i + 1), 0.0])
        log[-1]['update'] = [_i(ids[:2]), [0.3 * (i + 1), 0.0]]
    out.append({'seed': seed, 'priorities': prios, 'log': log})
  # distribution-level: probabilities of a fixed sample
  rs = np.random.RandomState(3)
  d = replay.PrioritizedDistribution(0.8, 0.1, rs, 0, None)
  d.add_priorities([2, 3, 5, 7], [1.0, 0.0, 3.0, 0.5])
  d.update_priorities([3], [4.0])
  d.remove_priorities([7])
  ids, probs = d.sample(6)
  dist = {'ops': [['add', [2, 3, 5, 7], [1.0, 0.0, 3.0, 0.5]],
                  ['update', [3], [4.0]], ['remove', [7]]],
          'seed': 3, 'exponent': 0.8, 'usp': 0.1, 'ids': _i(ids),
          'probs': _f(probs)}
  iw = replay.importance_sampling_weights(np.array([0.1, 0.25, 0.05, 0.6]),
                                          0.25, 0.4, True)
  return {'replay': out, 'distribution': dist,
          'is_weights': {'probs': [0.1, 0.25, 0.05, 0.6], 'uniform': 0.25,
                         'exponent': 0.4, 'weights': _f(iw)}}


def circular_cases(rc):
  out = {}
  # CircularLogitBuffer: add (log-mean-exp default) / popleft / setitem / sample
  rng = np.random.default_rng(11)
  b = rc.CircularLogitBuffer(6, rng)
  ops = []
  for v in (None, 1.5, None, -0.5, None, 2.0):
    b.add(v)
    ops.append(['add', v, _f(b._logits)])
  b.popleft()
  ops.append(['popleft', None, _f(b._logits)])
  b.add()
  ops.append(['add', None, _f(b._logits)])
  b[np.array([0, 2])] = np.array([0.25, -1.0], np.float32)
  ops.append(['setitem', [[0, 2], [0.25, -1.0]], _f(b._logits)])
  idx = b.sample(5)
  uni = b.sample_uniform(4, replace=False)
  out['logit_buffer'] = {'capacity': 6, 'seed': 11, 'ops': ops,
                         'left_head': b._left_head, 'sample': _i(idx),
                         'sample_uniform': _i(uni)}
  # MGSCFiFoTransitionReplay end to end
  rng = np.random.default_rng(4)
  r = rc.MGSCFiFoTransitionReplay(5, rc.Transition(None, None, None, None, None), rng)
  for i in range(8):
    r.add(rc.Transition(i, 0, 0.0, 1.0, i))
  s = r.sample(5)
  ind, tr, lg = r.batch_of_ids_transitions_and_logits(3)
  r.update_priorities(ind, np.array([0.5, -0.25, 1.0], np.float32))
  s2 = r.sample(4)
  out['mgsc_fifo'] = {'capacity': 5, 'seed': 4, 'n_add': 8,
                      'sample_items': _i(s.s_tm1), 'meta_indices': _i(ind),
                      'meta_items': _i(tr.s_tm1), 'meta_logits': _f(lg),
                      'sample2_items': _i(s2.s_tm1),
                      'logits': _f(r._distribution._logits)}
  # MGSCReservoirTransitionReplay
  rng = np.random.default_rng(9)
  r = rc.MGSCReservoirTransitionReplay(6, rc.Transition(None, None, None, None, None), rng)
  for i in range(20):
    r.add(rc.Transition(i, 0, 0.0, 1.0, i))
  logits_a = _f(r._distribution._logits)
  s = r.sample(5)
  ind, tr, lg = r.batch_of_ids_transitions_and_logits(3)
  r.update_priorities(ind, np.array([1.0, 0.0, -2.0], np.float32))
  s2 = r.sample(5)
  out['mgsc_reservoir'] = {'capacity': 6, 'seed': 9, 'n_add': 20,
                           'logits_after_adds': logits_a,
                           'slot_items': [int(x.s_tm1) for x in r._storage],
                           'sample_items': _i(s.s_tm1), 'meta_indices': _i(ind),
                           'meta_logits': _f(lg), 'sample2_items': _i(s2.s_tm1),
                           'logits': _f(r._distribution._logits)}
  return out


def main():
  replay, rc = _load_reference()
  golden = {
      'generator': 'tests/golden/make_golden.py (reference replay.py / '
                   'replay_circular.py, numpy %s)' % np.__version__,
      'sumtree': sumtree_cases(replay),
      'uniform_replay': uniform_replay_cases(replay),
      'reservoir': reservoir_cases(replay, rc),
      'prioritized': prioritized_cases(replay),
      'circular': circular_cases(rc),
  }
  with open(OUT, 'w') as f:
    json.dump(golden, f, indent=1)
  print('wrote', OUT)


if __name__ == '__main__':
  main()
