#!/bin/bash
# measure_policy's clock settle: 0 / 100 / 300 ms after 2 s idle, twice each.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05ba}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "
import json,time,torch,bench
d=torch.device('cuda:0')
for rep in range(2):
    for s in (0.0,100.0,300.0):
        time.sleep(2.0)
        r=bench.measure_policy(d,4096,settle_ms=s)
        print(json.dumps({'settle_ms':s,'act_ms':r['ms_per_step'],'bb_ms':r['backbone_roofline']['kernel_ms'],'bb_frac':r['backbone_roofline']['frac'],'settle':r['clock_settle']}),flush=True)
" > $OUT/settle.log 2>&1; echo rc=$?
grep '^{' $OUT/settle.log
