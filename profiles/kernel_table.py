"""Prints the libdqz kernels of a rocprofv3 --stats kernel_stats.csv."""
import csv
import re
import sys


def short(name):
  m = re.search(r'dqz::(\w+_kernel)', name)
  if not m:
    return None
  k = m.group(1)
  if k == 'multi_gemm_kernel':
    ops = re.findall(r'dqz::(\w+)(?:<[^>]*>)?', name)
    ops = [o for o in ops if o not in ('multi_gemm_kernel', 'Cfg', 'NoOp')]
    k = 'gemm[' + '+'.join(ops) + ']'
  return k


rows = []
for r in csv.DictReader(open(sys.argv[1])):
  s = short(r['Name'])
  if s:
    rows.append((s, int(r['Calls']), float(r['AverageNs']) / 1e3,
                 float(r['TotalDurationNs']) / 1e3))
tot = 0.0
for s, c, avg, total in sorted(rows, key=lambda x: -x[3]):
  print('%-48s calls %6d  avg %8.2f us' % (s, c, avg))
