#!/bin/bash
tail -2 gpurun_out/t1.log
for f in on off; do python -c "
import json;d=json.load(open('gpurun_out/bench_$f.json'));print('$f',d['value'],{k:round(v*1000,2) for k,v in d['phase_ms'].items()})"; done
grep -v amdgpu.ids gpurun_out/trace.txt
