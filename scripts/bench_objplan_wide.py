#!/usr/bin/env python3
"""Object plans (hbec_plan_objects: data and parity in separate arenas) with
k > 8, device-resident: every object goes through gf_apply_unaligned_plan
records, one launch per pass (8+3 for comparison takes the tiled kernel).
One JSON line per shape.

    python scripts/bench_objplan_wide.py
"""
import json, statistics, sys, torch
from pathlib import Path; sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from hummingbird_amd import batch as B, reedsolomon as RS
torch.cuda.set_device(0)
def t(fn, reps=9):
    fn(); ts=[]
    for _ in range(reps):
        a,b=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True); a.record(); fn(); b.record(); b.synchronize(); ts.append(a.elapsed_time(b))
    return statistics.median(ts)
for k,m,s in [(10,4,104864),(12,4,87392),(8,3,131072)]:
    n=2048
    d=torch.empty((n,k*s),dtype=torch.uint8,device='cuda'); B.fill_splitmix(d,k*s)
    p=torch.empty((n,m*s),dtype=torch.uint8,device='cuda')
    enc=RS.New(k,m)
    plan=B.StripePlan(enc, objects=[(d.data_ptr()+i*d.stride(0), p.data_ptr()+i*p.stride(0), s) for i in range(n)])
    ms=t(plan.encode); nb=n*(k+m)*s
    print(json.dumps({"k":k,"m":m,"n":n,"shard_len":s,"layout":"object plan (data + parity arenas)","encode_ms":round(ms,4),"frac":round(nb/ms/1e6/8000,4)}))
