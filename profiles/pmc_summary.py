"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch).
usage: python profiles/pmc_summary.py gpurun_out/pmc_<tag> [out.json]

HBM traffic per dispatch follows MI355X_MICROARCH.md (HBM section): the
FETCH_SIZE / WRITE_SIZE passes run separately; FETCH_SIZE (KB) counts 64 B
per 128-B request on gfx950, so it is doubled; WRITE_SIZE (KB) is taken as
is.  traffic_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
"""
import collections
import csv
import glob
import os
import json
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, 'p*', 'run_counter_collection.csv'))):
  for r in csv.DictReader(open(f)):
    name = r['Kernel_Name']
    if 'dqz' not in name:
      continue
    key = name.split('(')[0]
    key = key.replace('void dqz::multi_gemm_kernel<dqz::', '').replace('dqz::', '')[:70]
    vals[key][r['Counter_Name']].append(float(r['Counter_Value']))
    dur[key].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
for k, d in vals.items():
  m = {c: sum(v) / len(v) for c, v in d.items()}
  us = sum(dur[k]) / len(dur[k]) / 1e3
  print('%-70s %7.2fus' % (k, us))
  line = []
  for c in sorted(m):
    line.append('%s=%.4g' % (c, m[c]))
  wc = m.get('SQ_WAVE_CYCLES')
  if wc:
    for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY'):
      if c in m:
        line.append('%s/WC=%.2f' % (c, m[c] / wc))
  if 'GRBM_GUI_ACTIVE' in m:
    line.append('clk_GHz~%.2f' % (m['GRBM_GUI_ACTIVE'] / 8 / (us * 1e3)))
  print('   ' + ' '.join(line))

if len(sys.argv) > 2:
  out = {}
  for k, d in vals.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    short = k.split('<')[0].replace('void ', '').strip()
    rec = {'us': sum(dur[k]) / len(dur[k]) / 1e3}
    rec.update(m)
    if 'FETCH_SIZE' in m and 'WRITE_SIZE' in m:
      rec['traffic_bytes'] = 2 * m['FETCH_SIZE'] * 1024 + m['WRITE_SIZE'] * 1024
    out[short] = rec
  json.dump(out, open(sys.argv[2], 'w'), indent=1, sort_keys=True)

