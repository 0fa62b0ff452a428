"""Which kernels' ISA differs between two `hipcc --cuda-device-only -S`
outputs of learner.hip (basic-block labels normalised, so only instruction
changes count).  usage: python tools/isa_diff.py OLD.s NEW.s"""
import re
import sys


def kernels(path):
  out, cur = {}, None
  for line in open(path):
    m = re.match(r'^(_Z\w+):', line)
    if m:
      cur = m.group(1)
      out[cur] = []
      continue
    if cur is None:
      continue
    if line.strip().startswith(('.Lfunc_end', '; -- End')):
      cur = None
      continue
    line = re.sub(r'\.LBB\d+_\d+', 'L', line)
    out[cur].append(re.sub(r'BB\d+_\d+', 'BB', line))
  return out


def main():
  a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
  print('only in old:', [k for k in a if k not in b])
  print('only in new:', [k for k in b if k not in a])
  same = [k for k in a if k in b and a[k] == b[k]]
  print('identical: %d' % len(same))
  print('differ:', [k for k in a if k in b and a[k] != b[k]])


if __name__ == '__main__':
  main()
