"""Memory / MFMA / barrier instruction runs of one kernel in a hipcc -S file.

usage: python tools/isa_mem.py <file.s> <kernel-symbol-prefix>
Prints runs such as `13 buffer_load_dwordx4 | 17 s_waitcnt | ...`, to check
that a block's loads are in flight together (no load issued after an early
wait)."""
import itertools
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
start = next(i for i, l in enumerate(lines) if l.startswith(sys.argv[2] + ':'))
ins = []
for l in lines[start:]:
  l = l.strip()
  if re.match(r'(buffer_load|global_load|s_waitcnt vmcnt|s_barrier|s_sleep|v_mfma|global_store|buffer_store)', l):
    ins.append(l.split()[0])
  if 's_endpgm' in l:
    break
print(' | '.join('%d %s' % (len(list(g)), k) for k, g in itertools.groupby(ins)))
