#!/bin/bash
# Does the shard pitch (S) set the databuf encode rate?  8+3 at power-of-two,
# 16-B-aligned off-power-of-two and odd S, databuf and split (plan) layouts.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
S="c:8:3:131072:enc,c:8:3:131088:enc,c:8:3:133120:enc,c:8:3:139264:enc,c:8:3:131071:enc,c:8:3:131087:enc,c:8:3:133119:enc,c:8:3:139263:enc,c:8:3:131072:plan,c:8:3:133120:plan,c:8:3:131071:plan,c:8:3:133119:plan"
bash scripts/ab_odd.sh gpurun_out/r5_pitch.jsonl "$S" hummingbird_amd/libhbec.so
