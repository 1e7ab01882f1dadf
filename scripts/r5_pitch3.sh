#!/bin/bash
# Layout vs kernel at the slow pitch: 8+3 S = 131071 (and neighbours) as a
# strided databuf batch, as an object plan over the same databuf rows, and as
# an object plan with parity in its own array; table vs bit-plane strided.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
S=""
for s in 131071 131087 131199 133119; do S="$S,c:8:3:$s:enc,c:8:3:$s:dplan,c:8:3:$s:plan"; done
bash scripts/ab_odd.sh gpurun_out/r5_pitch3.jsonl "${S#,}" hummingbird_amd/libhbec.so tune_build/tune/libhbec.so:HBEC_ODD_BP=2
