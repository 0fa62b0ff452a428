"""Per-kernel average durations split by grid size from a rocprofv3
kernel-trace CSV (one row per dispatch), plus the sequence of one call.
usage: python tools/kernel_split.py <run_kernel_trace.csv> [name-filter]
"""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
flt = sys.argv[2] if len(sys.argv) > 2 else 'dqz'
agg = collections.defaultdict(list)
for r in rows:
  n = r['Kernel_Name']
  if flt not in n:
    continue
  key = (n.split('(')[0].replace('void ', '').replace('dqz::', '')[:40], int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']))
  agg[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for (n, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
  print('%-42s blocks %6d n %5d avg %8.2f us' % (n, g, len(v), sum(v) / len(v)))
