"""Per-kernel ISA counters of libdqz (integer-division expansions, float
divisions, vmcnt(0) drains, loads, MFMAs).  usage: python tools/isa_stats.py"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(tempfile.gettempdir(), 'dqz_isa.s')
subprocess.check_call(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '--cuda-device-only', '-S',
                       '-I' + os.path.join(ROOT, 'include'), '-o', out,
                       os.path.join(ROOT, 'dqn_mgsc_zoo_amd', 'csrc', 'learner.hip')], stderr=subprocess.DEVNULL)
stats, cur = {}, None
for line in open(out):
  m = re.match(r'^(_Z\w+):', line)
  if m:
    cur = m.group(1)
    stats[cur] = dict(lines=0, loads=0, vmcnt0=0, idiv=0, fdiv=0, mfma=0)
    continue
  if cur is None:
    continue
  st = stats[cur]
  st['lines'] += 1
  st['loads'] += ('global_load' in line) or ('buffer_load' in line)
  st['vmcnt0'] += 's_waitcnt vmcnt(0)' in line
  st['idiv'] += 'v_rcp_iflag' in line
  st['fdiv'] += 'v_div_scale' in line
  st['mfma'] += 'v_mfma' in line
  if 's_endpgm' in line:
    cur = None
filt = sys.argv[1] if len(sys.argv) > 1 else ''
for k, v in stats.items():
  name = subprocess.run(['c++filt', k], capture_output=True, text=True).stdout.strip()
  if filt in name:
    print('%-58s %s' % (name.split('(')[0][:58], ' '.join('%s=%d' % kv for kv in v.items())))
