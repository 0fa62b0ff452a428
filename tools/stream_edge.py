"""Cost of a hipGraph fork/join whose side branch finishes early (GPU box).

Graph of N iterations of 8 dependent tiny kernels on the main stream; variant
'fork' also forks a tiny side-stream kernel after kernel 2 and joins it
before kernel 7.  Prints us per iteration for each variant.
"""
import time
import torch

dev = torch.device('cuda:0')
x = torch.zeros(1024, device=dev)
y = torch.zeros(1024, device=dev)
main = torch.cuda.Stream(dev)
side = torch.cuda.Stream(dev)
N = 50


def body(fork, side_kernels):
  for i in range(8):
    if fork and i == 2:
      e = torch.cuda.Event()
      e.record(main)
      side.wait_event(e)
      with torch.cuda.stream(side):
        for _ in range(side_kernels):
          y.add_(1.0)
      e2 = torch.cuda.Event()
      e2.record(side)
    if fork and i == 7:
      main.wait_event(e2)
    x.add_(1.0)


def run(fork, side_kernels=1):
  with torch.cuda.stream(main):
    for _ in range(3):
      body(fork, side_kernels)
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g, stream=main):
    for _ in range(N):
      body(fork, side_kernels)
  for _ in range(5):
    g.replay()
  torch.cuda.synchronize()
  t = time.perf_counter()
  R = 40
  for _ in range(R):
    g.replay()
  torch.cuda.synchronize()
  return (time.perf_counter() - t) / (R * N) * 1e6


for rep in range(2):
  print('plain  %.2f us/iter' % run(False))
  print('fork1  %.2f us/iter' % run(True, 1))
  print('fork3  %.2f us/iter' % run(True, 3))
