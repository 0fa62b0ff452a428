"""ctypes binding of libdqz.so, the C ABI declared in include/dqz.h.

This is the only way the package reaches the device hot path.  There is no
CPU fallback: if the shared library is missing or fails to load, every
product entry point raises `NativeLibraryError`.
"""

import ctypes
import glob
import hashlib
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('DQZ_LIB') or os.path.join(_HERE, 'libdqz.so')
HEADER_PATH = os.path.join(os.path.dirname(_HERE), 'include', 'dqz.h')

DQZ_OK = 0
ALGO_DQN = 0
ALGO_DOUBLE = 1
ALGO_PER = 2
NUM_LEAVES = 10
NUM_PHASES = 10
# dqz_learner_profile's phase slots; slots 7 and 8 are merged into
# bwd_bc_kernel and report 0.
PHASE_NAMES = (
    'conv1_fwd', 'conv2_fwd', 'conv3_fwd', 'fc1_fwd', 'head', 'fc1_dx',
    'conv3_dx+conv2_dx+fc1_dw+conv3_dw+conv2_dw+conv1_dw', 'unused7',
    'unused8', 'update')
FRAME_H = 84
FRAME_W = 84
STACK = 4
FRAME_BYTES = FRAME_H * FRAME_W


class NativeLibraryError(RuntimeError):
  """libdqz.so is missing, failed to load, or a call returned an error."""


class DqzStore(ctypes.Structure):
  _fields_ = [
      ('frames', ctypes.c_void_p),
      ('fidx', ctypes.c_void_p),
      ('action', ctypes.c_void_p),
      ('reward', ctypes.c_void_p),
      ('discount', ctypes.c_void_p),
      ('capacity', ctypes.c_int64),
      ('num_frames', ctypes.c_int64),
  ]


class DqzParams(ctypes.Structure):
  _fields_ = [
      ('online', ctypes.c_void_p),
      ('target', ctypes.c_void_p),
      ('mu', ctypes.c_void_p),
      ('nu', ctypes.c_void_p),
  ]


class DqzLearnerConfig(ctypes.Structure):
  _fields_ = [
      ('batch', ctypes.c_int),
      ('num_actions', ctypes.c_int),
      ('algo', ctypes.c_int),
      ('learning_rate', ctypes.c_float),
      ('decay', ctypes.c_float),
      ('eps', ctypes.c_float),
      ('grad_error_bound', ctypes.c_float),
  ]


class DqzMetaConfig(ctypes.Structure):
  _fields_ = [
      ('meta_batch', ctypes.c_int),
      ('num_actions', ctypes.c_int),
      ('learning_rate', ctypes.c_float),
      ('decay', ctypes.c_float),
      ('eps', ctypes.c_float),
      ('grad_error_bound', ctypes.c_float),
      ('meta_learning_rate', ctypes.c_float),
      ('b1', ctypes.c_float),
      ('b2', ctypes.c_float),
      ('meta_eps', ctypes.c_float),
      ('second_order', ctypes.c_int),
  ]


class DqzAction(ctypes.Structure):
  _fields_ = [('action', ctypes.c_int32), ('value', ctypes.c_float)]


class DqzTransitionPut(ctypes.Structure):
  _fields_ = [
      ('slot', ctypes.c_int64),
      ('fidx', ctypes.c_int32 * 8),
      ('action', ctypes.c_int32),
      ('reward', ctypes.c_float),
      ('discount', ctypes.c_float),
      ('num_frames', ctypes.c_int32),
      ('frame_rows', ctypes.c_int32 * 8),
  ]


class DqzPerDraw(ctypes.Structure):
  _fields_ = [
      ('tree', ctypes.c_void_p),
      ('cap', ctypes.c_int64),
      ('live_base', ctypes.c_int64),
      ('size', ctypes.c_int64),
      ('capacity', ctypes.c_int64),
      ('uniform_sample_probability', ctypes.c_double),
      ('importance_sampling_exponent', ctypes.c_double),
      ('normalize_weights', ctypes.c_int),
      ('seed', ctypes.c_uint64),
      ('counter_dev', ctypes.c_void_p),
      ('injected_uniform', ctypes.c_void_p),
      ('injected_u', ctypes.c_void_p),
      ('index_to_slot', ctypes.c_void_p),
      ('alpha', ctypes.c_double),
      ('max_seen_dev', ctypes.c_void_p),
      ('out_indices', ctypes.c_void_p),
      ('out_slots', ctypes.c_void_p),
      ('out_probs', ctypes.c_void_p),
      ('out_weights', ctypes.c_void_p),
  ]


# name -> (restype, argtypes); must match include/dqz.h exactly.
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
SIGNATURES = {
    'dqz_last_error': (ctypes.c_char_p, []),
    'dqz_build_id': (ctypes.c_char_p, []),
    'dqz_param_layout': (
        _int,
        [_int, _int, ctypes.POINTER(_i64), ctypes.POINTER(_i64),
         ctypes.POINTER(_i64)],
    ),
    'dqz_learner_create': (
        _int, [ctypes.POINTER(DqzLearnerConfig), ctypes.POINTER(_vp)]),
    'dqz_learner_destroy': (_int, [_vp]),
    'dqz_learner_step': (
        _int,
        [_vp, ctypes.POINTER(DqzParams), ctypes.POINTER(DqzStore), _vp, _vp,
         _vp],
    ),
    'dqz_learner_step_uniform': (
        _int,
        [_vp, ctypes.POINTER(DqzParams), ctypes.POINTER(DqzStore), _i64, _i64,
         _i64, ctypes.c_uint64, _vp, _vp, _vp],
    ),
    'dqz_learner_step_per': (
        _int,
        [_vp, ctypes.POINTER(DqzParams), ctypes.POINTER(DqzStore), _vp, _vp,
         _vp, _i64, _vp, ctypes.c_double, _vp, _vp]),
    'dqz_learner_step_logits': (
        _int,
        [_vp, ctypes.POINTER(DqzParams), ctypes.POINTER(DqzStore), _vp, _vp,
         ctypes.c_uint64, _vp, _vp, _vp, _vp]),
    'dqz_learner_step_per_draw': (
        _int,
        [_vp, ctypes.POINTER(DqzParams), ctypes.POINTER(DqzStore),
         ctypes.POINTER(DqzPerDraw), _vp]),
    'dqz_learner_grad': (
        _int,
        [_vp, ctypes.POINTER(DqzParams), ctypes.POINTER(DqzStore), _vp, _vp,
         _vp, _vp],
    ),
    'dqz_learner_outputs': (_int, [_vp, _vp, _vp, _vp, _vp]),
    'dqz_learner_sync_status': (_int, [_vp, _vp]),
    'dqz_learner_debug_stall': (_int, [_vp, _int, ctypes.c_uint]),
    'dqz_per_write_back': (_int, [_vp, _vp, _i64, _vp, ctypes.c_double, _vp, _vp]),
    'dqz_learner_profile': (
        _int,
        [_vp, ctypes.POINTER(DqzParams), ctypes.POINTER(DqzStore), _vp, _vp,
         _int, ctypes.POINTER(ctypes.c_float), _vp],
    ),
    'dqz_forward': (_int, [_vp, _vp, _vp, _int, _vp, _vp]),
    'dqz_forward_slots': (
        _int, [_vp, _vp, ctypes.POINTER(DqzStore), _vp, _int, _int, _vp, _vp]),
    'dqz_act': (
        _int, [_vp, _vp, _vp, _int, ctypes.c_double, ctypes.c_uint64,
               ctypes.c_uint64, _vp, _vp]),
    'dqz_store_put': (
        _int, [ctypes.POINTER(DqzStore), ctypes.POINTER(DqzTransitionPut), _vp,
               _vp]),
    'dqz_frame_plan_create': (_int, [_int, _int, _int, _int, ctypes.POINTER(_vp)]),
    'dqz_frame_plan_destroy': (_int, [_vp]),
    'dqz_atari_frame': (_int, [_vp, _vp, _int, _vp, _vp]),
    'dqz_sample_uniform': (
        _int, [_i64, _i64, _i64, _int, ctypes.c_uint64, _vp, _vp, _vp]),
    'dqz_gather_stacks': (
        _int, [ctypes.POINTER(DqzStore), _vp, _int, _int, _vp, _vp]),
    'dqz_target_copy': (_int, [_vp, _vp, _i64, _vp]),
    'dqz_logit_buffer_create': (_int, [_i64, _int, ctypes.POINTER(_vp)]),
    'dqz_logit_buffer_destroy': (_int, [_vp]),
    'dqz_logits_add': (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp]),
    'dqz_logits_sample': (_int, [_vp, _vp, _vp, _int, _vp, _vp]),
    'dqz_logits_sample_slots': (
        _int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, _int, _vp, _vp, _vp]),
    'dqz_logits_sample_exact': (_int, [_vp, _vp, _vp, _int, _vp, _vp, _vp]),
    'dqz_logits_add_exact': (_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _vp]),
    'dqz_logits_probs': (_int, [_vp, _vp, _vp, _vp, _vp]),
    'dqz_logits_terms': (_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    'dqz_logits_write': (_int, [_vp, _vp, _vp, _vp, _int, _vp]),
    'dqz_logits_put': (_int, [_vp, _vp, _i64, ctypes.c_float, _vp]),
    'dqz_logits_invalidate': (_int, [_vp]),
    'dqz_logits_run_get': (
        _int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_float),
               ctypes.POINTER(_int), ctypes.POINTER(_int), ctypes.POINTER(_int), _vp]),
    'dqz_logits_run_set': (
        _int, [_vp, _vp, ctypes.c_double, ctypes.c_float, _int, _int, _int, _vp]),
    'dqz_uniform_philox': (_int, [ctypes.c_uint64, _vp, _int, _vp, _vp]),
    'dqz_sumtree_set': (_int, [_vp, _i64, _vp, _vp, _int, _vp]),
    'dqz_sumtree_query': (_int, [_vp, _i64, _vp, _int, _vp, _vp]),
    'dqz_per_sample': (
        _int,
        [_vp, _i64, _i64, _i64, _i64, _int, ctypes.c_double, ctypes.c_double,
         _int, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'dqz_per_add': (
        _int,
        [_vp, _i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, _vp,
         ctypes.c_double, _vp, ctypes.c_int32, _vp]),
    'dqz_meta_create': (
        _int, [ctypes.POINTER(DqzMetaConfig), ctypes.POINTER(_vp)]),
    'dqz_meta_destroy': (_int, [_vp]),
    'dqz_meta_update': (
        _int,
        [_vp, ctypes.POINTER(DqzParams), ctypes.POINTER(DqzStore), _vp,
         ctypes.POINTER(DqzStore), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'dqz_meta_outputs': (_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    'dqz_meta_sync_status': (_int, [_vp, _vp]),
    'dqz_meta_debug_stall': (_int, [_vp, _int, ctypes.c_uint]),
}

_lib = None
_lock = threading.Lock()


def source_files():
  """The files a libdqz.so is compiled from: csrc/*.hip, csrc/*.hpp, dqz.h."""
  files = sorted(glob.glob(os.path.join(_HERE, 'csrc', '*.hip')) +
                 glob.glob(os.path.join(_HERE, 'csrc', '*.hpp')))
  return files + [HEADER_PATH]


def source_build_id():
  """First 16 hex digits of SHA-256 over the library's sources on disk.

  __graft_entry__.build() bakes this into the library (dqz_build_id); lib()
  refuses a library whose id differs, so a GPU run cannot silently test a
  stale binary.
  """
  h = hashlib.sha256()
  for f in source_files():
    h.update(os.path.basename(f).encode() + b'\0')
    with open(f, 'rb') as fh:
      h.update(fh.read())
    h.update(b'\0')
  return h.hexdigest()[:16]


def build_id():
  """The id baked into the loaded library."""
  return lib().dqz_build_id().decode()


def lib():
  """Loads libdqz.so once; raises NativeLibraryError if it is unavailable."""
  global _lib
  if _lib is not None:
    return _lib
  with _lock:
    if _lib is None:
      if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            '%s not found: build it with `python -c "import __graft_entry__ '
            'as g; g.build()"` (hipcc --offload-arch=gfx950).' % LIB_PATH)
      try:
        handle = ctypes.CDLL(LIB_PATH)
      except OSError as e:
        raise NativeLibraryError('failed to load %s: %s' % (LIB_PATH, e)) from e
      for name, (restype, argtypes) in SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = restype
        fn.argtypes = argtypes
      got, want = handle.dqz_build_id().decode(), source_build_id()
      # DQZ_ALLOW_STALE=1 is for tools/abv.sh A/Bs of prebuilt variants only.
      if got != want and os.environ.get('DQZ_ALLOW_STALE') != '1':
        raise NativeLibraryError(
            '%s was built from other sources (build id %s, sources on disk %s):'
            ' rebuild it with `python -c "import __graft_entry__ as g; '
            'g.build()"`.' % (LIB_PATH, got, want))
      _lib = handle
  return _lib


def check(rc):
  """Raises NativeLibraryError with dqz_last_error() on a non-zero status."""
  if rc != DQZ_OK:
    msg = lib().dqz_last_error()
    raise NativeLibraryError(
        'libdqz error %d: %s' % (rc, msg.decode() if msg else ''))
  return rc


def param_layout(num_actions, shared_bias):
  """Returns (offsets, sizes, total) of the flat parameter buffer."""
  offs = (_i64 * NUM_LEAVES)()
  sizes = (_i64 * NUM_LEAVES)()
  total = _i64()
  check(lib().dqz_param_layout(
      int(num_actions), int(bool(shared_bias)), offs, sizes,
      ctypes.byref(total)))
  return list(offs), list(sizes), int(total.value)


def ptr(t):
  """Device pointer of a torch tensor (None -> NULL)."""
  if t is None:
    return None
  return ctypes.c_void_p(t.data_ptr())


def stream_handle(stream=None):
  import torch  # pylint: disable=g-import-not-at-top
  s = stream if stream is not None else torch.cuda.current_stream()
  return ctypes.c_void_p(s.cuda_stream)
