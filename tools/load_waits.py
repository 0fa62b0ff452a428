"""Flags kernels whose loads before the first barrier are split by vmcnt
waits (a load issued after a wait costs an extra memory round trip).
usage: python tools/load_waits.py [asm.s]   (builds the device asm if omitted)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1:
  path = sys.argv[1]
else:
  path = os.path.join(tempfile.gettempdir(), 'dqz_waits.s')
  subprocess.check_call(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '--cuda-device-only',
                         '-S', '-I' + os.path.join(ROOT, 'include'), '-o', path,
                         os.path.join(ROOT, 'dqn_mgsc_zoo_amd', 'csrc', 'learner.hip')], stderr=subprocess.DEVNULL)
cur, seen_barrier, waited, late = None, False, False, {}
for line in open(path):
  m = re.match(r'^(_Z\w+):', line)
  if m:
    cur, seen_barrier, waited = m.group(1), False, False
    late[cur] = 0
    continue
  if cur is None or seen_barrier:
    continue
  if 's_barrier' in line:
    seen_barrier = True
  elif re.search(r's_waitcnt.*vmcnt', line):
    waited = True
  elif ('global_load' in line or 'buffer_load' in line) and waited:
    late[cur] += 1
for k, v in late.items():
  if v:
    name = subprocess.run(['c++filt', k], capture_output=True, text=True).stdout.strip().split('(')[0]
    print('%-50s loads issued after a vmcnt wait (before 1st barrier): %d' % (name, v))
