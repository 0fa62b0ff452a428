"""CPU: libdqz.so loads and exports every function include/dqz.h declares,
and the ctypes binding table matches the header (no compute calls)."""

import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'dqz.h')


def _declared():
  text = open(HEADER).read()
  text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
  return sorted(set(re.findall(r'\b(dqz_\w+)\s*\(', text)))


@pytest.fixture(scope='module')
def libdqz():
  from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
  if not os.path.exists(_native.LIB_PATH):
    import __graft_entry__  # pylint: disable=g-import-not-at-top
    __graft_entry__._compile_lib()  # pylint: disable=protected-access
  return ctypes.CDLL(_native.LIB_PATH)


def test_header_declares_the_abi():
  names = _declared()
  assert 'dqz_learner_step' in names and 'dqz_meta_update' in names
  assert len(names) >= 25


def test_library_exports_every_declared_symbol(libdqz):
  missing = [n for n in _declared() if not hasattr(libdqz, n)]
  assert not missing, missing


def test_binding_table_matches_header(libdqz):
  from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
  assert sorted(_native.SIGNATURES) == _declared()
  _native.lib()  # binds restype/argtypes of every symbol


def test_error_paths_without_a_gpu(libdqz):
  """Argument validation runs before any HIP call."""
  from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
  lib = _native.lib()
  offs = (ctypes.c_int64 * 10)()
  sizes = (ctypes.c_int64 * 10)()
  total = ctypes.c_int64()
  assert lib.dqz_param_layout(6, 0, offs, sizes, ctypes.byref(total)) == 0
  assert sum(sizes) == 1687206 and total.value % 64 == 0
  assert lib.dqz_param_layout(6, 1, offs, sizes, ctypes.byref(total)) == 0
  assert sum(sizes) == 1687201
  assert lib.dqz_param_layout(0, 0, offs, sizes, ctypes.byref(total)) == -1
  assert b'num_actions' in lib.dqz_last_error()
  cfg = _native.DqzLearnerConfig(0, 6, 0, 2.5e-4, 0.95, 1e-5, 1 / 32)
  h = ctypes.c_void_p()
  assert lib.dqz_learner_create(ctypes.byref(cfg), ctypes.byref(h)) == -1
  assert b'batch' in lib.dqz_last_error()
  mcfg = _native.DqzMetaConfig(0, 6, 2.5e-4, 0.95, 1e-5, 1 / 32, 2.5e-4,
                               0.9, 0.999, 1e-8)
  assert lib.dqz_meta_create(ctypes.byref(mcfg), ctypes.byref(h)) == -1
  with pytest.raises(_native.NativeLibraryError, match='meta_batch'):
    _native.check(lib.dqz_meta_create(ctypes.byref(mcfg), ctypes.byref(h)))


def test_bench_prices_every_reportable_phase():
  """Every phase name dqz_learner_profile can report has the algorithmic
  FLOPs, bytes and kernel symbol bench.py's roofline needs."""
  import sys  # pylint: disable=g-import-not-at-top
  sys.path.insert(0, ROOT)
  import bench  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
  names = set(_native.PHASE_NAMES) - {'unused7', 'unused8'}
  for algo in ('dqn', 'double'):
    flops, nbytes = bench.phase_flops(algo, 32), bench.phase_bytes(algo, 32)
    for n in names:
      assert n in flops and n in nbytes and n in bench.PHASE_KERNEL, n
      assert nbytes[n] > 0, n
  # the launches together count each FLOP of the step once (conv_fwd is the
  # one launch of conv1..conv3, reported instead of their three phases)
  for algo in ('dqn', 'double'):
    f = bench.phase_flops(algo, 32)
    assert f['conv_fwd'] == f['conv1_fwd'] + f['conv2_fwd'] + f['conv3_fwd']
    assert sum(v for k, v in f.items() if k != 'conv_fwd') == bench.STEP_FLOP[algo]


def test_library_build_id_matches_sources(libdqz):
  """The loaded libdqz.so was compiled from the sources on disk."""
  from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
  assert libdqz.dqz_build_id  # exported
  assert _native.build_id() == _native.source_build_id()
  assert len(_native.source_build_id()) == 16


def test_stale_library_is_refused(monkeypatch):
  """lib() raises when the library's id differs from the sources."""
  from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
  saved = _native._lib  # pylint: disable=protected-access
  try:
    monkeypatch.setattr(_native, '_lib', None)
    monkeypatch.setattr(_native, 'source_build_id', lambda: '0' * 16)
    monkeypatch.delenv('DQZ_ALLOW_STALE', raising=False)
    with pytest.raises(_native.NativeLibraryError, match='other sources'):
      _native.lib()
  finally:
    _native._lib = saved  # pylint: disable=protected-access
