"""Per-kernel means of rocprofv3 --pmc CSVs, one directory per library.
usage: python tools/pmc_by_dir.py gpurun_out/<tag>   (reads <tag>/p_*/...csv)"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
keys = sys.argv[2:] or ['fwd_conv_kernel<1>', 'bwd_bc_kernel<false>', 'fc1_fwd32', 'head_kernel', 'fc1_dx', 'update_kernel']
for d in sorted(glob.glob(os.path.join(root, 'p_*'))):
  files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
  if not files:
    continue
  vals = collections.defaultdict(lambda: collections.defaultdict(list))
  for f in files:
    for r in csv.DictReader(open(f)):
      vals[r['Kernel_Name'].split('(')[0].replace('void dqz::', '').replace('dqz::', '')][r['Counter_Name']].append(
          float(r['Counter_Value']))
  print('==', os.path.basename(d))
  for k, c in vals.items():
    if not any(x in k for x in keys):
      continue
    m = {n: sum(v) / len(v) for n, v in c.items()}
    lds, conf = m.get('SQ_INSTS_LDS', 0), m.get('SQ_LDS_BANK_CONFLICT', 0)
    print('  %-34s LDS %9.0f conflicts %9.0f (%.3f/instr) waitLDS %.3g VALU %.3g MFMA %.3g' % (
        k[:34], lds, conf, conf / lds if lds else 0, m.get('SQ_WAIT_INST_LDS', 0), m.get('SQ_INSTS_VALU', 0),
        m.get('SQ_INSTS_VALU_MFMA_F32', 0)))
