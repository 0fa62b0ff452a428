"""Per-kernel durations of a profiles/run_profile.sh kernel trace, split into
the hipGraph replays and the back-to-back profile launches.

usage: python profiles/trace_split.py gpurun_out/prof_<tag>/run_kernel_trace.csv [eager] [profile_iters]

run_profile.sh runs bench.py with 3 eager warm-up steps (graph capture
prologue), then 1,100 graph-replayed steps, then `profile_iters` (20)
back-to-back launches of every phase; each kernel's dispatches are taken
in start order and cut at those counts.
"""
import collections
import csv
import re
import sys

path = sys.argv[1]
eager = int(sys.argv[2]) if len(sys.argv) > 2 else 3
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rows = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
  m = re.search(r'dqz::(\w+_kernel)', r['Kernel_Name'])
  if m:
    rows[m.group(1)].append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
print('%-22s %6s %9s %9s' % ('kernel', 'n', 'graph_us', 'b2b_us'))
for k, v in sorted(rows.items()):
  v.sort()
  d = [(e - s) / 1e3 for s, e in v]
  g, p = d[eager:len(d) - reps], d[len(d) - reps:]
  print('%-22s %6d %9.2f %9.2f' % (k, len(d), sum(g) / max(1, len(g)), sum(p) / max(1, len(p))))
