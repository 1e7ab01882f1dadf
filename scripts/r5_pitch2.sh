#!/bin/bash
# Fine sweep of the shard pitch: 8+3 databuf encode at S = 2^17 + 16 j (aligned
# kernel) and S = 2^17 - 1 + 16 j (record kernel), j = 0..15.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
S=""
for j in $(seq 0 15); do S="$S,c:8:3:$((131072 + 16 * j)):enc,c:8:3:$((131071 + 16 * j)):enc"; done
bash scripts/ab_odd.sh gpurun_out/r5_pitch2.jsonl "${S#,}" hummingbird_amd/libhbec.so
