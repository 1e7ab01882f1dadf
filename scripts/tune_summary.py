import json, sys
for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tune.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"{d['variant']:12s} enc {d['enc_ms_med']:.4f}/{d['enc_ms_min']:.4f} rec {d['rec_ms_med']:.4f}/{d['rec_ms_min']:.4f} "
              f"GB/s {d['enc_GBs']:7.1f} {d['rec_GBs']:7.1f} frac {d['frac']:.4f} ok={d['parity_ok'] and d['rebuilt_ok']} "
              f"tile={d.get('tile')} bpc={d.get('blocks_per_cu')}")
