# Host-path encode + ShardHash (bench_host.py step 13: 4096 x 1 MiB, 4+2 and
# 8+3, pageable and pinned) over hash-arena count / size and hash ordering.
set -e
mkdir -p gpurun_out
for cfg in "2 1024 -" "2 2048 -" "2 3072 -" "2 3072 1" "2 3072 0" "4 512 1" "2 1024 0"; do
  set -- $cfg
  echo "{\"arenas\": $1, \"arena_mb\": $2, \"serial\": \"$3\"}" >> gpurun_out/md5arenas.jsonl
  if [ "$3" = "-" ]; then unset HBEC_MD5_SERIAL; else export HBEC_MD5_SERIAL=$3; fi
  HBEC_HASH_ARENAS=$1 HBEC_HASH_ARENA_MB=$2 timeout -k 10 200 python scripts/bench_host.py 13 >> gpurun_out/md5arenas.jsonl 2>&1
done
