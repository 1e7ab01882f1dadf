# Zero-copy stripes kernel grid cap (HBEC_ZC_GRID): host encode of 4096 x 1 MiB
# pinned stripes (bench_host.py 4), 262 144 x 4 KiB stripes (14), and
# encode + ShardHash (13).  Two passes over the caps.
set -e
mkdir -p gpurun_out
for pass in 1 2; do
  for g in 0 128 64 32; do
    echo "{\"zc_grid\": $g, \"pass\": $pass}" >> gpurun_out/zcgrid.jsonl
    HBEC_ZC_GRID=$g timeout -k 10 200 python scripts/bench_host.py 4 13 14 >> gpurun_out/zcgrid.jsonl 2>&1
  done
done
