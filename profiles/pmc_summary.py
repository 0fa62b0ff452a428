"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch).
usage: python profiles/pmc_summary.py gpurun_out/pmc_<tag>"""
import collections
import csv
import glob
import os
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
