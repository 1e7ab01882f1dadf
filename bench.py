#!/usr/bin/env python3
"""Headline benchmark: device-resident 4+2 EC encode + reconstruct of batched
1 MiB objects on MI355X (BASELINE.json metric, configs[1] + configs[2]).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

One step = one pass of the hot path over one batch held in HBM:
  1. Encoder.Encode   of 4096 objects x 1 MiB  (4 data shards read, 2 parity written)
  2. Encoder.Reconstruct of the same 4096 objects with shards {0,1} erased
     (survivors 2,3,P0,P1 read, the 2 data shards written)
Per object the algorithmic traffic of each op is k*S read + 2*S written =
1.5 MiB, 12 GiB per step per GPU.  `value` = algorithmic bytes
of all ranks / max-over-ranks time, in GiB/s.  Objects are partitioned across
ranks (rank r owns global objects [r*4096, (r+1)*4096)): weak scaling, no
data-path collective; torch.distributed carries only the barrier and the
max-time reduction.

Extra objects on the JSON line: `roofline` (dominant kernel = the
gf_apply_vec_pipe2<4,2> kernel that both ops launch, as `dispatches_per_op`
dispatches of 1024 objects each (tuning.h HBEC_VEC_CHUNK_TILES); achieved =
algorithmic bytes per op / the op's HIP-event-timed average duration on the
launch stream, i.e. the summed dispatch times plus the gaps between them;
traffic = PMC HBM bytes per dispatch from the committed rocprofv3 summary
profiles/*_pmc.json times the dispatches per op, used only when that file was
collected on the kernel sources being run -- same sha256 -- else null), `cpu_baseline`
(oracle/gf_oracle.c's AVX2 port of klauspost's algorithm over the host cores
on a bounded sample, rank 0 at N=1) and `config5` (BASELINE configs[4]: a
65 536 x 1 MiB 4+2 batch partitioned contiguously over the N ranks, encoded
device-resident, at every N including 1) and `small_objects` (the reference
README's 4 KB shape: 65 536 x 4 KiB objects, 8+3 and 4+2, Encode /
Reconstruct / Verify, rank 0) and `config4` (BASELINE configs[3]: 8+3 over
mixed 4 KiB / 1 MiB objects, one object-plan launch per op, rank 0).

`--gpus N` without a launcher (WORLD_SIZE unset) starts N rank processes
itself through torch.distributed.run, before this process touches the GPU;
a launcher whose WORLD_SIZE differs from --gpus is refused.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402
from hummingbird_amd import split as SP  # noqa: E402

METRIC = "GiB/s device-resident EC encode+reconstruct, 4+2 @ 1 MiB; % HBM roofline"
GiB = float(1 << 30)
MiB = 1 << 20
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
KERNEL_NAME = "gf_apply_vec_pipe2<4, 2>"


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def partition(n_per_rank: int, rank: int) -> tuple[int, int]:
    """Global object range [first, first+n) owned by `rank` (weak scaling)."""
    return rank * n_per_rank, n_per_rank


def max_over_ranks(pg, values, device):
    """Element-wise max of a list of floats over all ranks (the only
    collective in the bench: control, not data path)."""
    if pg is None:
        return list(values)
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return t.tolist()


def gather_ranks(pg, values, device):
    """Every rank's list of floats, in rank order (control traffic only)."""
    if pg is None:
        return [list(values)]
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(pg.get_world_size())]
    pg.all_gather(out, t)
    return [o.tolist() for o in out]


# Sources whose compiled code the dominant kernel is (gf_apply_vec_pipe2 and
# its device helpers): a PMC summary is only reported as this run's traffic
# when it was collected on exactly these sources.
KERNEL_SOURCES = ("hummingbird_amd/csrc/kernels.hip", "hummingbird_amd/csrc/gf_device.h",
                  "hummingbird_amd/csrc/kernels.h", "hummingbird_amd/csrc/tuning.h")


def kernel_sources_sha256(sources=KERNEL_SOURCES) -> str:
    h = hashlib.sha256()
    for rel in sources:
        h.update(rel.encode())
        h.update((ROOT / rel).read_bytes())
    return h.hexdigest()


# Sources of the odd_objects legs' kernels (gf_odd_rec / gf_odd of 4+2, 8+3,
# 10+4 and gf_odd_edges): their traffic is reported only from a PMC summary
# collected on exactly these sources (pmc_summary.py records both hashes).
ODD_SOURCES = ("hummingbird_amd/csrc/odd.hip", "hummingbird_amd/csrc/odd_impl.h", "hummingbird_amd/csrc/gf_device.h",
               "hummingbird_amd/csrc/kernels.h", "hummingbird_amd/csrc/odd_k58.hip", "hummingbird_amd/csrc/odd_k912.hip",
               "hummingbird_amd/csrc/tuning.h", "hummingbird_amd/csrc/odd_bp.hip", "hummingbird_amd/csrc/xor_sched.h")


def vec_chunk_tiles() -> int:
    """Tiles per launch of the aligned strided kernels (tuning.h
    HBEC_VEC_CHUNK_TILES): a batch runs as launches of whole objects."""
    for line in (ROOT / "hummingbird_amd/csrc/tuning.h").read_text().splitlines():
        parts = line.split()
        if len(parts) >= 3 and parts[0] == "#define" and parts[1] == "HBEC_VEC_CHUNK_TILES":
            return int(parts[2])
    raise RuntimeError("HBEC_VEC_CHUNK_TILES not in tuning.h")


def load_pmc(prefix_glob="profiles/r[0-9][0-9]_pmc.json"):
    """Latest committed PMC summary, if it was collected on the kernel
    sources of this tree; (data, path, reason_if_rejected)."""
    files = sorted(glob.glob(str(ROOT / prefix_glob)))
    if not files:
        return None, None, "no PMC summary under profiles/"
    data = json.loads(Path(files[-1]).read_text())
    rel = os.path.relpath(files[-1], ROOT)
    want = kernel_sources_sha256()
    got = data.get("kernel_sources_sha256")
    if got != want:
        return None, rel, f"stale: {rel} was collected on kernel sources {str(got)[:12]}, this tree is {want[:12]}"
    return data, rel, None


# PMC attribution: before each leg that quotes PMC traffic, one fill_splitmix
# launch of exactly PMC_MARK_BLOCKS + i blocks (i = the leg's index in
# PMC_LEGS) marks where that leg's dispatches begin, so scripts/pmc_summary.py
# can give each leg the bytes of its own launches (two legs launching the same
# kernel, e.g. the random-size and mid-size plans, are no longer averaged)
PMC_LEGS = ("odd_objects", "random_objects", "mid_objects")
PMC_MARK_BLOCKS = 9001
_mark_buf = []


def pmc_mark(leg):
    i = PMC_LEGS.index(leg)
    if not _mark_buf:
        _mark_buf.append(torch.empty((1, (PMC_MARK_BLOCKS + len(PMC_LEGS)) * 2048), dtype=torch.uint8, device="cuda"))
    nb = (PMC_MARK_BLOCKS + i) * 2048  # 256 threads x 8 B per block
    B.fill_splitmix(_mark_buf[0][:, :nb], nb)


def pmc_kernels(pmc, leg):
    """The per-kernel PMC bytes of one leg's own launches (pmc_summary.py
    `legs`); {} when the summary predates the markers."""
    return (pmc or {}).get("legs", {}).get(leg, {})


class Workload:
    """4+2 batch resident in HBM: objs [n, 1 MiB], parity [n, 512 KiB],
    rebuilt [n, 512 KiB] (reconstruct target for the erased shards 0,1)."""

    def __init__(self, k, m, n, obj_len, first, erased):
        self.k, self.m, self.n, self.obj_len = k, m, n, obj_len
        self.s = obj_len // k
        self.erased = list(erased)
        self.enc = RS.New(k, m)
        self.objs = torch.empty((n, obj_len), dtype=torch.uint8, device="cuda")
        self.parity = torch.empty((n, m * self.s), dtype=torch.uint8, device="cuda")
        self.rebuilt = torch.empty((n, len(self.erased) * self.s), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(self.objs, obj_len, first=first)
        self.enc_views = B.shard_views(self.objs, k, self.s) + B.shard_views(self.parity, m, self.s)
        rv = list(self.enc_views)
        for slot, i in enumerate(self.erased):
            rv[i] = (self.rebuilt.data_ptr() + slot * self.s, self.rebuilt.stride(0))
        self.rec_views = rv
        self.present = [0 if i in self.erased else 1 for i in range(k + m)]
        # algorithmic bytes per launch: k*S read + (m | e)*S written per object
        self.enc_bytes = n * (k + m) * self.s
        self.rec_bytes = n * (k + len(self.erased)) * self.s

    def encode(self):
        B.encode_views(self.enc, self.enc_views, self.n, self.s)

    def reconstruct(self):
        B.reconstruct_views(self.enc, self.rec_views, self.present, self.n, self.s)

    def verify(self) -> bool:
        torch.cuda.synchronize()
        want = torch.cat([self.objs[:, i * self.s:(i + 1) * self.s] for i in self.erased], dim=1)
        return bool(torch.equal(self.rebuilt, want))


def cpu_baseline(k, m, obj_len, erased, budget_s=12.0, sample_objs=512, gpu=None):
    """Oracle AVX2 port over the host threads, bounded sample, same two ops.
    gpu: (objects, parity, rebuilt) of the timed headline batch's first
    sample_objs objects (host copies, taken after the timed region); the CPU
    sample is the same splitmix objects, so the oracle's parity and rebuilt
    shards are compared with the GPU's byte for byte (`oracle_match`)."""
    import numpy as np

    from oracle import coracle as CO
    from oracle import oracle as O

    threads = CO.cpu_threads()
    s = obj_len // k
    objs = CO.fill_objects(0, sample_objs, obj_len)
    parity = np.empty((sample_objs, m * s), dtype=np.uint8)
    rebuilt = np.empty((sample_objs, len(erased) * s), dtype=np.uint8)
    mat = CO.build_matrix(k, m)
    enc_in = [(objs.ctypes.data + j * s, obj_len) for j in range(k)]
    enc_out = [(parity.ctypes.data + r * s, m * s) for r in range(m)]
    present = [0 if i in erased else 1 for i in range(k + m)]
    surv, inv = O.Encoder(k, m).decode_matrix(present)
    rows = [inv[i] for i in erased]
    all_views = enc_in + enc_out
    rec_in = [all_views[i] for i in surv]
    rec_out = [(rebuilt.ctypes.data + e * s, len(erased) * s) for e in range(len(erased))]
    t_total, passes = 0.0, 0
    while t_total < budget_s or passes == 0:
        t_total += CO.apply_batch(mat[k:], enc_in, enc_out, sample_objs, s, threads)
        t_total += CO.apply_batch(rows, rec_in, rec_out, sample_objs, s, threads)
        passes += 1
        if passes >= 20000:
            break
    assert np.array_equal(rebuilt, np.concatenate([objs[:, i * s:(i + 1) * s] for i in erased], axis=1))
    match = None
    if gpu is not None:
        g_objs, g_par, g_reb = gpu
        match = bool(np.array_equal(g_objs, objs) and np.array_equal(g_par, parity) and np.array_equal(g_reb, rebuilt))
    nbytes = passes * sample_objs * ((k + m) * s + (k + len(erased)) * s)
    # single thread, same two ops, bounded (~2 s)
    t1, p1 = 0.0, 0
    while t1 < 2.0 and p1 < 2000:
        t1 += CO.apply_batch(mat[k:], enc_in, enc_out, 32, s, 1)
        t1 += CO.apply_batch(rows, rec_in, rec_out, 32, s, 1)
        p1 += 1
    single = p1 * 32 * ((k + m) * s + (k + len(erased)) * s) / t1 / GiB
    # config 1: one object through an ecSplit-shaped call, single thread, with
    # the per-call New + (k+m)*chunk alloc ecSplit does (ecutils.go:27,31-35)
    # and kernel-only
    one = objs[0].copy()
    reps = sorted(CO.ecsplit_once(k, m, one, MiB, CO.AVX2, True) for _ in range(100))
    reps_k = sorted(CO.ecsplit_once(k, m, one, MiB, CO.AVX2, False) for _ in range(100))
    return {
        "value": round(nbytes / t_total / GiB, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{passes} passes x {sample_objs} x 1 MiB objects, encode + reconstruct{{{','.join(map(str, erased))}}}, "
                  f"{t_total:.1f} s wall, AVX2 nibble-table port of klauspost galMulAVX2Xor "
                  f"(oracle/gf_oracle.c), {threads} threads, {cpu_model()}",
        "single_thread_GiB_s": round(single, 3),
        "config1_ecsplit_1mib_single_thread_ms": round(reps[len(reps) // 2] * 1e3, 4),
        "config1_kernel_only_single_thread_ms": round(reps_k[len(reps_k) // 2] * 1e3, 4),
        "oracle_match": match,
        "oracle_match_sample": (f"objects 0..{sample_objs - 1} of the timed batch: GPU parity and rebuilt shards "
                                f"{{{','.join(map(str, erased))}}} vs the oracle's, byte for byte") if gpu is not None else None,
    }


def batch_split(pg, k, m, obj_len, n_global, world, rank, ctl_device):
    """BASELINE configs[4]: a 4+2 batch of n_global objects lands on rank 0's
    GPU; it is scattered over xGMI (RCCL P2P, hummingbird_amd/split.py), every
    rank encodes its partition, and the parity is gathered back to rank 0,
    which checks it against its own encode of the whole batch.  Runs after the
    headline measurement; its times are reported next to it, never in `value`."""
    s = obj_len // k
    first, n = SP.object_range(n_global, world, rank)
    enc = RS.New(k, m)
    device = "cuda"
    batch = dest = want = part = parity = None
    err = ""
    try:  # allocate everything first; all ranks agree before any P2P starts
        if rank == 0:
            batch = torch.empty((n_global, obj_len), dtype=torch.uint8, device=device)
            B.fill_splitmix(batch, obj_len)
            dest = torch.empty((n_global, m * s), dtype=torch.uint8, device=device)
            want = torch.empty_like(dest)
        part = torch.empty((n, obj_len), dtype=torch.uint8, device=device)
        parity = torch.empty((n, m * s), dtype=torch.uint8, device=device)
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 - reported, and every rank skips together
        err = f"rank {rank}: {type(e).__name__}: {e}"[:200]
    (failed,) = max_over_ranks(pg, [1.0 if err else 0.0], ctl_device)
    if failed:
        return {"skipped": err or "allocation failed on another rank", "objects": n_global}

    def timed(fn):
        pg.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        pg.barrier()
        return time.perf_counter() - t

    t_sc = timed(lambda: SP.scatter_objects(pg, batch, part, n_global))
    t_enc = timed(lambda: B.encode_objects(enc, part, parity, s))
    t_ga = timed(lambda: SP.gather_rows(pg, parity, dest, n_global))
    ok = 1.0
    if rank == 0:  # the gathered parity must equal rank 0's own encode of the whole batch
        B.encode_objects(enc, batch, want, s)
        for a in range(0, n_global, 1024):  # chunked: torch.equal materialises a bool temp
            if not torch.equal(want[a:a + 1024], dest[a:a + 1024]):
                ok = 0.0
                break
    t_sc, t_enc, t_ga, bad = max_over_ranks(pg, [t_sc, t_enc, t_ga, 1.0 - ok], ctl_device)
    peer_objs = n_global - SP.object_range(n_global, world, 0)[1]
    sc_bytes = peer_objs * obj_len
    ga_bytes = peer_objs * m * s
    return {
        "backend": "rccl (torch.distributed nccl, P2P over xGMI)",
        "objects": n_global, "objects_per_rank_max": SP.object_range(n_global, world, 0)[1],
        "scatter_ms": round(t_sc * 1e3, 3), "scatter_GBs": round(sc_bytes / t_sc / 1e9, 2),
        "scatter_GBs_per_peer": round(sc_bytes / max(1, world - 1) / t_sc / 1e9, 2),
        "encode_ms": round(t_enc * 1e3, 3),
        "encode_GiB_s_all_ranks": round(n_global * (k + m) * s / t_enc / GiB, 2),
        "gather_ms": round(t_ga * 1e3, 3), "gather_GBs": round(ga_bytes / t_ga / 1e9, 2),
        "end_to_end_ms": round((t_sc + t_enc + t_ga) * 1e3, 3),
        "parity_ok": bad == 0.0,
    }


def config5(pg, k, m, obj_len, n_global, world, rank, ctl_device, reps=3):
    """BASELINE configs[4] at this N: n_global objects partitioned
    contiguously over the ranks (rank r owns SP.object_range(n_global, world,
    r)), each rank's partition generated in and encoded from its own HBM (no
    data-path collective: objects are independent, ecutils.go:38-70).  At
    N=1 that is 64 GiB of objects + 32 GiB of parity on one GPU.  `reps`
    encodes of the whole partition are timed between barriers; the parity is
    then checked on the GPU by Encoder.Verify (gf_verify_pipe, a different
    kernel from the encoder)."""
    s = obj_len // k
    first, n = SP.object_range(n_global, world, rank)
    enc = RS.New(k, m)
    objs = parity = flags = None
    err = ""
    try:
        objs = torch.empty((n, obj_len), dtype=torch.uint8, device="cuda")
        parity = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        B.fill_splitmix(objs, obj_len, first=first)
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 - reported; every rank skips together
        err = f"rank {rank}: {type(e).__name__}: {e}"[:200]
    (failed,) = max_over_ranks(pg, [1.0 if err else 0.0], ctl_device)
    if failed:
        return {"skipped": err or "allocation failed on another rank", "objects": n_global}
    B.encode_objects(enc, objs, parity, s)  # warm-up
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    if pg:
        pg.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e0, e1 in ev:
        e0.record(stream)
        B.encode_objects(enc, objs, parity, s)
        e1.record(stream)
    torch.cuda.synchronize()
    if pg:
        pg.barrier()
    elapsed = time.perf_counter() - t0
    launch_ms = sum(a.elapsed_time(b) for a, b in ev) / reps
    B.verify_views(enc, B.shard_views(objs, k, s) + B.shard_views(parity, m, s), n, s, flags)
    bad = float(int(flags.count_nonzero().item()))
    elapsed, launch_ms, bad = max_over_ranks(pg, [elapsed, launch_ms, bad], ctl_device)
    del objs, parity, flags
    torch.cuda.empty_cache()
    n_max = SP.object_range(n_global, world, 0)[1]
    per_gpu_gbs = n_max * (k + m) * s / (launch_ms * 1e-3) / 1e9
    return {
        "workload": f"{k}+{m} Encode of {n_global} x {obj_len >> 20} MiB objects partitioned contiguously over "
                    f"{world} GPU(s) (BASELINE configs[4]), device-resident",
        "objects": n_global, "objects_per_gpu_max": n_max, "reps": reps,
        "ms": round(elapsed / reps * 1e3, 3),
        "value_GiB_s": round(n_global * (k + m) * s * reps / elapsed / GiB, 2),
        "per_gpu_launch_ms_max": round(launch_ms, 3),
        "per_gpu_roofline": {"achieved": round(per_gpu_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(per_gpu_gbs / HBM_PEAK_GBS, 4)},
        "parity_ok": bad == 0.0,
        "parity_check": "Encoder.Verify on the GPU (gf_verify_pipe), every object",
    }


def small_objects(n=65536, obj_len=4096, reps=100, settle=200):
    """The reference README's 4 KB shape (/root/reference/README.md:19-27)
    device-resident: n x 4 KiB objects, 8+3 (512-B shards) and 4+2 (1 KiB),
    Encode, Reconstruct of the first m data shards and Verify, each timed over
    `reps` back-to-back launches with HIP events on the launch stream.
    Algorithmic bytes per object: (k+m)*S for Encode and Verify, (k+e)*S for
    Reconstruct.  Rebuilt shards are compared with the
    originals and Verify must pass every object.  `settle` launches run
    first: over the first ~10 ms of sustained short launches the GPU's clocks
    dip and recover (8+3 @ 4 KiB: 65 % -> 56 % -> 72 % of 8 TB/s over ~150
    launches, profiles/r02_small_dvfs_drift.jsonl), and a shorter warm-up
    times the dip, not the kernel."""
    out = {"workload": f"{n} x {obj_len} B objects, device-resident (README 4 KB shape)", "shapes": []}
    stream = torch.cuda.current_stream()
    for k, m in ((8, 3), (4, 2)):
        s = obj_len // k
        miss = list(range(m))
        enc = RS.New(k, m)
        objs = torch.empty((n, obj_len), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(objs, obj_len, first=1 << 20)
        par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
        rebuilt = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        views = B.shard_views(objs, k, s) + B.shard_views(par, m, s)
        rv = list(views)
        for slot, i in enumerate(miss):
            rv[i] = (rebuilt.data_ptr() + slot * s, rebuilt.stride(0))
        present = [0 if i in miss else 1 for i in range(k + m)]
        ops = {
            "encode": (lambda: B.encode_views(enc, views, n, s), n * (k + m) * s),
            "reconstruct": (lambda: B.reconstruct_views(enc, rv, present, n, s), n * (k + m) * s),
            "verify": (lambda: B.verify_views(enc, views, n, s, flags), n * (k + m) * s),
        }
        row = {"k": k, "m": m, "shard_bytes": s, "kernel_kind": B.kernel_info(k, m, s)["kind"]}
        for _ in range(settle):
            ops["encode"][0]()
        for name, (fn, nbytes) in ops.items():
            for _ in range(10):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            gbs = nbytes / (ms * 1e-3) / 1e9
            row[name] = {"ms": round(ms, 5), "GB_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
        ok = int(flags.count_nonzero()) == 0
        for slot, i in enumerate(miss):
            ok = ok and torch.equal(rebuilt[:, slot * s:(slot + 1) * s], objs[:, i * s:(i + 1) * s])
        row["parity_ok"] = bool(ok)
        out["shapes"].append(row)
        del objs, par, rebuilt, flags
    torch.cuda.empty_cache()
    return out


def _route_delta(fn):
    """Run fn once and return which odd-shard kernel families it launched
    (B.odd_path_stats() after minus before)."""
    p0 = B.odd_path_stats()
    fn()
    torch.cuda.synchronize()
    p1 = B.odd_path_stats()
    return {x: p1[x] - p0[x] for x in p1}


def _odd_kernel_traffic(kern, k, r, mode, paths, plan=False):
    """PMC bytes per launch of the odd-shard kernel that coded (k, r, mode),
    chosen by the route the leg actually took (`paths`, from _route_delta):
    the bit-plane instance gf_odd_rec<k, r, mode, XS, LIST> (XS >= 0), the
    table record instance (XS = -1), or the strided gf_odd<k, r, mode>; LIST =
    plans' tile-list instance.  None when the summary holds no instance, or
    more than one, of the family that ran."""
    pre = f"gf_odd_rec<{k}, {r}, {mode}, "
    tail = "true>" if plan else "false>"
    recs = sorted(x for x in kern if x.startswith(pre) and x.endswith(tail))
    if paths.get("bitplane", 0) > 0:
        pick = [x for x in recs if not x.startswith(pre + "-1,")]
    elif paths.get("records", 0) > 0:
        pick = [x for x in recs if x.startswith(pre + "-1,")]
    elif paths.get("strided", 0) > 0 and not plan:
        pick = [x for x in (f"gf_odd<{k}, {r}, {mode}>",) if x in kern]
    else:
        pick = []
    if len(pick) != 1:
        return None, None
    return pick[0], kern[pick[0]].get("hbm_bytes_per_launch")


def odd_leg(k, m, n, obj_len, first, reps=20, settle=40, kern=None):
    """One odd-shard shape: n ecSplit databufs of obj_len-byte objects,
    device-resident: Encode, Reconstruct of shards {0,1} in place, Verify.
    Rebuilt shards must equal the originals and Verify must pass every object."""
    s = -(-obj_len // k)
    enc = RS.New(k, m)
    rows = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(rows, (k + m) * s, first=first)
    views = B.shard_views(rows, k + m, s)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    present = [0, 0] + [1] * (k + m - 2)
    nbytes = {"encode": n * (k + m) * s, "reconstruct": n * (k + 2) * s, "verify": n * (k + m) * s}
    stream = torch.cuda.current_stream()
    B.encode_views(enc, views, n, s)
    keep = rows[:, :2 * s].clone()
    ops = {"encode": lambda: B.encode_views(enc, views, n, s),
           "reconstruct": lambda: B.reconstruct_views(enc, views, present, n, s),
           "verify": lambda: B.verify_views(enc, views, n, s, flags)}
    out = {"workload": f"{k}+{m}, {n} ecSplit databufs of {obj_len} B objects (S = {s}, shards at odd offsets), "
                       "device-resident", "shard_bytes": s}
    for _ in range(settle):
        ops["encode"]()
    routes = {}
    for name, fn in ops.items():
        routes[name] = _route_delta(fn)
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gbs = nbytes[name] / (ms * 1e-3) / 1e9
        out[name] = {"ms": round(ms, 4), "GB_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                     "edges": "fused" if routes[name]["fused"] > 0 else "separate launch"}
    if kern:
        for name, (r, mode) in (("encode", (m, 0)), ("reconstruct", (2, 0)), ("verify", (m, 2))):
            kname, t = _odd_kernel_traffic(kern, k, r, mode, routes[name])
            # the edge kernel when the guard bands took their own launch (a
            # batch of >= kOddEdgeSplitObjs objects: one thread per slot, all outputs)
            te = 0
            if routes[name]["edges"] > 0:
                te = kern.get("gf_odd_edges<2, false, 128>" if name == "verify" else "gf_odd_edges<0, false, 128>",
                              {}).get("hbm_bytes_per_launch")
                t = None if te is None else t
            if t is not None:
                out[name]["kernel"] = kname
                out[name]["traffic"] = int(t + (te or 0))
                out[name]["traffic_ratio"] = round((t + (te or 0)) / nbytes[name], 4)
    # the check: erase shards 0-1 of every object for real, rebuild them, and
    # Verify every object (a reconstruct that wrote nothing would fail here)
    rows[:, :2 * s].fill_(0x3C)
    ops["reconstruct"]()
    flags.zero_()
    ops["verify"]()
    torch.cuda.synchronize()
    out["parity_ok"] = bool(int(flags.count_nonzero()) == 0 and torch.equal(rows[:, :2 * s], keep))
    del rows, keep, flags
    torch.cuda.empty_cache()
    return out


def odd_objects(n=4096):
    """Objects of arbitrary size: ecSplit's S = ceil(len / k) is a multiple of
    16 for one object size in 16 (objectserver/ecutils.go:14-24), and its
    databuf puts shard i at i*S (ecutils.go:31-35), so most objects reach the
    codec as shards at odd offsets.  The 4+2 leg (1 MiB - 4 B objects, S =
    262 143) at the top level; 8+3 (1 MiB - 8 B, S = 131 071: BASELINE
    configs[3]'s shape) and 10+4 (1 MiB, S = 104 858) under `shapes`.  HBM
    traffic per launch comes from the committed PMC summary (two --pmc passes
    over this bench) when it was collected on these sources."""
    pmc_files = sorted(glob.glob(str(ROOT / "profiles/r[0-9][0-9]_pmc.json")))
    pmc = json.loads(Path(pmc_files[-1]).read_text()) if pmc_files else {}
    fresh = pmc.get("odd_sources_sha256") == kernel_sources_sha256(ODD_SOURCES)
    kern = pmc_kernels(pmc, "odd_objects") if fresh else None
    pmc_mark("odd_objects")
    out = odd_leg(4, 2, n, (1 << 20) - 4, 1 << 21, kern=kern)
    out["shapes"] = {"8+3": odd_leg(8, 3, n, (1 << 20) - 8, 1 << 22, kern=kern),
                     "10+4": odd_leg(10, 4, n, 1 << 20, 1 << 23, kern=kern)}
    out["traffic_source"] = os.path.relpath(pmc_files[-1], ROOT) if (pmc_files and fresh) else None
    if not fresh:
        out["traffic_note"] = "no PMC summary collected on this tree's odd-kernel sources"
    out["parity_ok"] = out["parity_ok"] and all(v["parity_ok"] for v in out["shapes"].values())
    return out


def random_objects(n=4096, shapes=((4, 2), (8, 3)), reps=20, settle=40):
    """The nursery stabilizer's batch shape: a scan hands
    over the oldest nursery objects whatever their sizes (indexdb.go:26,548-557,
    ecengine.go:583-640), so S = ceil(len / k) (ecutils.go:14-24) takes many
    values.  n objects with seeded shard lengths uniform in [4 KiB / k,
    1 MiB / k], odd, as ONE object plan (data arena + parity arena,
    hbec_plan_objects): per-stripe records over the plan's tile list, one
    launch per pass.  Encode is timed; every object is then checked with the
    product's Verify (a different kernel family), and the -m gpu test
    (tests/test_gpu_random_plan.py) compares every object with the oracle.
    HBM traffic per launch from the committed PMC summary (main + edge +
    record kernels) when it was collected on these sources."""
    pmc_files = sorted(glob.glob(str(ROOT / "profiles/r[0-9][0-9]_pmc.json")))
    pmc = json.loads(Path(pmc_files[-1]).read_text()) if pmc_files else {}
    fresh = pmc.get("odd_sources_sha256") == kernel_sources_sha256(ODD_SOURCES)
    stream = torch.cuda.current_stream()
    out = {"workload": f"{n} objects, shard length uniform in [4 KiB/k, 1 MiB/k] and odd (seeded), one object "
                       "plan per shape, Encode, device-resident", "shapes": {}}
    kern = pmc_kernels(pmc, "random_objects") if fresh else {}
    pmc_mark("random_objects")
    for k, m in shapes:
        rng = __import__("numpy").random.default_rng(0x48424543 + 100 * k + m)
        sizes = [int(x) | 1 for x in rng.integers(4096 // k, (1 << 20) // k + 1, n)]
        data = torch.empty(sum(k * s for s in sizes), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(data.view(1, -1), data.numel(), first=11 * k + m)
        parity = torch.empty(sum(m * s for s in sizes), dtype=torch.uint8, device="cuda")
        objs, do, po = [], 0, 0
        for s in sizes:
            objs.append((data.data_ptr() + do, parity.data_ptr() + po, s))
            do += k * s
            po += m * s
        enc = RS.New(k, m)
        plan = B.StripePlan(enc, objects=objs)
        paths = _route_delta(plan.encode)
        for _ in range(settle):
            plan.encode()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            plan.encode()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        nbytes = sum((k + m) * s for s in sizes)
        gbs = nbytes / (ms * 1e-3) / 1e9
        flags = torch.zeros(1, dtype=torch.int32, device="cuda")
        bad = 0
        for (a_, b_, s) in objs:
            views = [(a_ + j * s, 0) for j in range(k)] + [(b_ + r * s, 0) for r in range(m)]
            B.verify_views(enc, views, 1, s, flags)
        torch.cuda.synchronize()
        bad = int(flags.item())
        leg = {"objects": n, "bytes": nbytes, "ms": round(ms, 4), "GB_s": round(gbs, 1),
               "frac": round(gbs / HBM_PEAK_GBS, 4), "parity_ok": bad == 0}
        leg["edges"] = "fused" if paths["fused"] > 0 else "separate launch"
        if kern:
            kname, t = _plan_traffic(kern, k, m, paths)
            if t is not None:
                leg["kernel"] = kname
                leg["traffic"] = int(t)
                leg["traffic_ratio"] = round(t / nbytes, 4)
        out["shapes"][f"{k}+{m}"] = leg
        del plan, data, parity, flags
        torch.cuda.empty_cache()
    out["traffic_source"] = os.path.relpath(pmc_files[-1], ROOT) if (pmc_files and fresh) else None
    out["parity_ok"] = all(v["parity_ok"] for v in out["shapes"].values())
    return out


def _plan_traffic(kern, k, r, paths):
    """PMC bytes per launch of a plan pass: the record kernel of the family
    that ran (`paths`, from _route_delta), the per-stripe record writer, and
    the guard-band kernel when the bands took their own launch."""
    kname, t = _odd_kernel_traffic(kern, k, r, 0, paths, plan=True)
    if t is None:
        return None, None
    extra = [kern.get("gf_odd_planrec", {}).get("hbm_bytes_per_launch")]
    if paths["edges"] > 0:
        extra.append(kern.get("gf_odd_edges_plan<0, false, 128>", {}).get("hbm_bytes_per_launch"))
    if any(x is None for x in extra):
        return None, None
    return kname, t + sum(extra)


def mid_objects(n=16384, shapes=((4, 2), (8, 3)), reps=20, settle=40):
    """Mid-size objects, the size class most object stores hold (VERDICT r05
    item 1): n objects with lengths log-uniform in [8 KiB, 128 KiB] (seeded),
    S = ceil(len / k) (ecutils.go:14-24) forced odd, so every shard sits at an
    odd offset.  Per shape, the same objects in two layouts, one plan each:
    ecSplit databufs back to back (hbec_plan_stripes: shard i at base + i S,
    ecutils.go:31-35) and an object plan (data arena + parity arena,
    hbec_plan_objects).  Encode is timed over `reps` launches after `settle`;
    every 16th object is then checked with the product's Verify, and the -m
    gpu tests compare such plans with the oracle byte for byte.  `aligned_32k`:
    the same n objects at exactly 32 KiB, 8+3 (S = 4096), as a strided batch
    (the packed kernel), Encode / Reconstruct {0,1,2} / Verify.  HBM traffic
    per launch from the committed PMC summary when it was collected on these
    sources."""
    import numpy as np

    pmc_files = sorted(glob.glob(str(ROOT / "profiles/r[0-9][0-9]_pmc.json")))
    pmc = json.loads(Path(pmc_files[-1]).read_text()) if pmc_files else {}
    fresh = pmc.get("odd_sources_sha256") == kernel_sources_sha256(ODD_SOURCES)
    kern = pmc_kernels(pmc, "mid_objects") if fresh else {}
    pmc_mark("mid_objects")
    stream = torch.cuda.current_stream()

    def timed(fn):
        for _ in range(settle):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    out = {"workload": f"{n} objects of log-uniform length in [8 KiB, 128 KiB], S = ceil(len/k) forced odd, "
                       "device-resident, Encode; ecSplit databufs (stripe plan) and data + parity arenas "
                       "(object plan)", "shapes": {}}
    for k, m in shapes:
        rng = np.random.default_rng(0x4D494430 + 100 * k + m)
        lens = np.exp(rng.uniform(np.log(8 << 10), np.log(128 << 10), n))
        sizes = [int(-(-int(x) // k)) | 1 for x in lens]
        nbytes = sum((k + m) * s for s in sizes)
        enc = RS.New(k, m)
        legs = {}
        for layout in ("databuf", "object_plan"):
            if layout == "databuf":
                arena = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
                B.fill_splitmix(arena.view(1, -1), arena.numel(), first=31 * k + m)
                stripes, off = [], 0
                for s in sizes:
                    stripes.append((arena.data_ptr() + off, s))
                    off += (k + m) * s
                plan = B.StripePlan(enc, stripes=stripes)
                views_of = [([(b + j * s, 0) for j in range(k + m)], s) for b, s in stripes]
                keep = (arena,)
            else:
                data = torch.empty(sum(k * s for s in sizes), dtype=torch.uint8, device="cuda")
                B.fill_splitmix(data.view(1, -1), data.numel(), first=37 * k + m)
                parity = torch.empty(sum(m * s for s in sizes), dtype=torch.uint8, device="cuda")
                objs, do, po = [], 0, 0
                for s in sizes:
                    objs.append((data.data_ptr() + do, parity.data_ptr() + po, s))
                    do += k * s
                    po += m * s
                plan = B.StripePlan(enc, objects=objs)
                views_of = [([(a + j * s, 0) for j in range(k)] + [(b + r * s, 0) for r in range(m)], s)
                            for a, b, s in objs]
                keep = (data, parity)
            paths = _route_delta(plan.encode)
            ms = timed(plan.encode)
            gbs = nbytes / (ms * 1e-3) / 1e9
            flags = torch.zeros(1, dtype=torch.int32, device="cuda")
            for views, s in views_of[::16]:
                B.verify_views(enc, views, 1, s, flags)
            torch.cuda.synchronize()
            leg = {"objects": n, "bytes": nbytes, "ms": round(ms, 4), "GB_s": round(gbs, 1),
                   "frac": round(gbs / HBM_PEAK_GBS, 4), "parity_ok": int(flags.item()) == 0,
                   "launches": paths}
            if kern:
                kname, t = _plan_traffic(kern, k, m, paths)
                if t is not None:
                    leg["kernel"] = kname
                    leg["traffic"] = int(t)
                    leg["traffic_ratio"] = round(t / nbytes, 4)
            legs[layout] = leg
            del plan, keep, flags
            torch.cuda.empty_cache()
        out["shapes"][f"{k}+{m}"] = legs
    # exact 32 KiB 8+3 objects (aligned S = 4096): a strided batch
    k, m, s = 8, 3, 4096
    enc = RS.New(k, m)
    objs = torch.empty((n, k * s), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * s, first=41)
    par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    rebuilt = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    views = B.shard_views(objs, k, s) + B.shard_views(par, m, s)
    rv = list(views)
    for slot in range(m):
        rv[slot] = (rebuilt.data_ptr() + slot * s, rebuilt.stride(0))
    present = [0] * m + [1] * k
    al = {"workload": f"{n} x 32 KiB objects, 8+3 (S = 4096), strided batch", "shard_bytes": s,
          "kernel_kind": B.kernel_info(k, m, s)["kind"]}
    for name, fn in (("encode", lambda: B.encode_views(enc, views, n, s)),
                     ("reconstruct", lambda: B.reconstruct_views(enc, rv, present, n, s)),
                     ("verify", lambda: B.verify_views(enc, views, n, s, flags))):
        ms = timed(fn)
        gbs = n * (k + m) * s / (ms * 1e-3) / 1e9
        al[name] = {"ms": round(ms, 4), "GB_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    ok = int(flags.count_nonzero()) == 0
    for slot in range(m):
        ok = ok and torch.equal(rebuilt[:, slot * s:(slot + 1) * s], objs[:, slot * s:(slot + 1) * s])
    al["parity_ok"] = bool(ok)
    out["aligned_32k"] = al
    del objs, par, rebuilt, flags
    torch.cuda.empty_cache()
    out["traffic_source"] = os.path.relpath(pmc_files[-1], ROOT) if (pmc_files and fresh) else None
    out["parity_ok"] = al["parity_ok"] and all(v["parity_ok"] for legs in out["shapes"].values()
                                               for v in legs.values())
    return out


def config4(n=4096, reps=20, settle=40):
    """BASELINE configs[3]: 8+3 Encode + Reconstruct{0,1,2} of n objects of
    4 KiB or 1 MiB (p = 0.5 each, by the splitmix64 byte stream of the base
    seed) in one launch per op through an object plan (data
    arena + parity arena, hbec_plan_objects).  Algorithmic
    bytes: (k+m)*S per object for Encode, (k+3)*S for Reconstruct.  Check:
    the reconstruct rebuilds shards 0-2 in place from the parity the encode
    wrote, and the data arena must come back byte for byte."""
    k, m, miss = 8, 3, (0, 1, 2)
    present = [0 if i in miss else 1 for i in range(k + m)]
    flags = torch.empty((1, n), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(flags, n)
    sizes = [MiB if int(b) & 1 else 4096 for b in flags.cpu()[0].tolist()]
    enc = RS.New(k, m)
    dl, pl, doff, poff = [], [], 0, 0
    for size in sizes:
        s = size // k
        dl.append((doff, s))
        pl.append(poff)
        doff += k * s
        poff += m * s
    data = torch.empty(doff, dtype=torch.uint8, device="cuda")
    parity = torch.empty(poff, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(data.view(1, -1), doff, first=7)
    want = data.clone()
    plan = B.StripePlan(enc, objects=[(data.data_ptr() + o, parity.data_ptr() + po, s)
                                      for (o, s), po in zip(dl, pl)])
    stream = torch.cuda.current_stream()
    for _ in range(settle):
        plan.encode()
    ms = {}
    for name, fn in (("encode", plan.encode), ("reconstruct", lambda: plan.reconstruct(present))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ms[name] = e0.elapsed_time(e1) / reps
    plan.encode()
    data[:dl[0][1] * 3].zero_()  # erase shards 0-2 of object 0 for real before the rebuild
    plan.reconstruct(present)
    torch.cuda.synchronize()
    ok = bool(torch.equal(data, want))
    enc_bytes = sum((k + m) * s for _, s in dl)
    rec_bytes = sum((k + len(miss)) * s for _, s in dl)
    total_ms = ms["encode"] + ms["reconstruct"]
    gbs = (enc_bytes + rec_bytes) / (total_ms * 1e-3) / 1e9
    n_big = sum(1 for x in sizes if x == MiB)
    del plan, data, parity, want
    torch.cuda.empty_cache()
    return {"workload": f"8+3 Encode + Reconstruct{{0,1,2}} of {n} objects, {n_big} x 1 MiB + {n - n_big} x 4 KiB "
                        "(BASELINE configs[3]), object plan, one launch per op, device-resident",
            "encode_ms": round(ms["encode"], 4), "reconstruct_ms": round(ms["reconstruct"], 4),
            "bytes_per_step": enc_bytes + rec_bytes, "GB_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "parity_ok": ok, "parity_check": "in-place rebuild of shards 0-2 from the encoded parity equals the data"}


def host_path(k, m, obj_len, n_obj=2048, passes=5, all_devices=False):
    """The path as the object server runs it: stripes (ecSplit databuf layout,
    ecutils.go:31-35) in pinned host memory from hbec_host_alloc, coded in
    place over PCIe by Encoder.EncodeStripes (zero-copy host path).  With
    all_devices, one process drives every visible GPU (hbec_encode_host_devices).
    PCIe-inclusive; reported beside `value`, never as it."""
    s = obj_len // k
    enc = RS.New(k, m)
    hb = RS.HostBuffer(n_obj * (k + m) * s)
    try:
        rows = hb.array.reshape(n_obj, (k + m) * s)
        dev = torch.empty((n_obj, obj_len), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(dev, obj_len)
        par = torch.empty((n_obj, m * s), dtype=torch.uint8, device="cuda")
        B.encode_objects(enc, dev, par, s)
        rows[:, :k * s] = dev.cpu().numpy()
        want = par.cpu().numpy()
        del dev, par
        stripes = [rows[i] for i in range(n_obj)]
        run = (lambda: enc.EncodeStripesDevices(stripes)) if all_devices else (lambda: enc.EncodeStripes(stripes))
        run()
        ok = bool((rows[:, k * s:] == want).all())
        ts = []
        for _ in range(passes):
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[len(ts) // 2]
        return {"op": "encode", "objects": n_obj, "memory": "pinned (hbec_host_alloc), zero-copy",
                "devices": RS.device_count() if all_devices else 1,
                "ms": round(t * 1e3, 3), "object_data_GiB_s": round(n_obj * obj_len / t / GiB, 2),
                "pcie_GB_s": round(n_obj * (k + m) * s / t / 1e9, 2), "parity_ok": ok}
    finally:
        hb.free()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown cpu"


def spawn_ranks(n: int, argv: list[str]) -> int:
    """`--gpus N` with no launcher: run this script as N ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) in a
    CHILD process and return its exit status.  The caller has not touched the
    GPU (nothing is exec'd from a process that initialised it)."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]
    return subprocess.run(cmd).returncode


def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle-ms", type=float, default=60.0,
                    help="untimed steps before the W warm-up steps until this much GPU time has passed, "
                         "so the clocks have left their start-up ramp (0 = none)")
    ap.add_argument("--objects", type=int, default=4096, help="objects per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-small", action="store_true",
                    help="skip the README 4 KB shape leg (small_objects) and the config4 leg")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the PCIe-inclusive host-path line (pinned stripes, zero-copy)")
    ap.add_argument("--config5-objects", type=int, default=65536,
                    help="BASELINE configs[4]: objects partitioned over the N GPUs (0 = skip)")
    ap.add_argument("--split-objects", type=int, default=65536,
                    help="N>1 on RCCL: objects in the batch split from rank 0 (BASELINE configs[4]); 0 = skip")
    ap.add_argument("--dry-run", action="store_true",
                    help="control path only (rank spawn, gloo rendezvous, max-over-ranks): no GPU, no value")
    return ap.parse_args(argv)


def dry_run(world, rank):
    """The N>1 control path without a GPU (tests/test_dist.py): every rank
    joins a gloo group and the max-over-ranks reduction; rank 0 reports how
    many ranks took part."""
    pg = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
        pg = dist
    (seen,) = max_over_ranks(pg, [float(rank + 1)], "cpu")
    per_rank = gather_ranks(pg, [float(rank), float(10 * rank)], "cpu")
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world,
                          "ranks_seen": int(seen), "per_rank": per_rank, "dry_run": True}), flush=True)
    if pg:
        pg.destroy_process_group()
    return 0


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, argv)
    world, rank, local = dist_env()
    if world != args.gpus:
        print(f"bench.py: launcher WORLD_SIZE={world} but --gpus {args.gpus}; refusing to report a "
              f"{world}-GPU number as {args.gpus}", file=sys.stderr)
        return 2
    if args.dry_run:
        return dry_run(world, rank)

    # one rank per GPU; HBEC_DIST_BACKEND=gloo lets several ranks share one
    # GPU to rehearse the N>1 path on a 1-GPU box (control traffic only)
    backend = os.environ.get("HBEC_DIST_BACKEND", "nccl")
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    pg = None
    ctl_device = "cuda" if backend == "nccl" else "cpu"
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        pg = dist

    k, m, obj_len, erased = 4, 2, MiB, (0, 1)
    first, n = partition(args.objects, rank)
    w = Workload(k, m, n, obj_len, first, erased)
    stream = torch.cuda.current_stream()

    # warm-up runs straight into the timed region: any idle gap here (e.g. a
    # verification pass loading torch's reduce kernels, ~0.2 s) lets the GPU
    # drop its clocks, and the next ~15 launches then ramp from 1.37 back to
    # 1.08 ms (kernel trace, profiles/r02_ramp_kernel_trace.txt).  The result
    # is verified after the timed region instead.
    # The clock ramp lasts ~10-14 launches (~15 ms); the driver's `--warmup 5`
    # is 10 launches, so untimed settle steps run first until --settle-ms of
    # GPU time has passed.  They are reported as `settle_steps`.
    settle_steps = 0
    if args.settle_ms > 0:
        t_settle = time.perf_counter()
        while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms and settle_steps < 1000:
            w.encode()
            w.reconstruct()
            settle_steps += 1
            if settle_steps % 4 == 0:
                torch.cuda.synchronize()
    for _ in range(args.warmup):
        w.encode()
        w.reconstruct()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if pg:
        pg.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        e0, e1, e2 = ev[i]
        e0.record(stream)
        w.encode()
        e1.record(stream)
        w.reconstruct()
        e2.record(stream)
    torch.cuda.synchronize()
    if pg:
        pg.barrier()
    elapsed = time.perf_counter() - t0
    ok = w.verify()

    enc_ms = sum(e0.elapsed_time(e1) for e0, e1, _ in ev) / args.steps
    rec_ms = sum(e1.elapsed_time(e2) for _, e1, e2 in ev) / args.steps
    per_rank = gather_ranks(pg, [enc_ms, rec_ms], ctl_device) if world > 1 else None
    elapsed, enc_ms, rec_ms, bad = max_over_ranks(pg, [elapsed, enc_ms, rec_ms, 0.0 if ok else 1.0], ctl_device)
    ok = bad == 0.0

    step_bytes = w.enc_bytes + w.rec_bytes
    total_bytes = step_bytes * args.steps * world
    value = total_bytes / elapsed / GiB
    ms_per_step = elapsed / args.steps * 1e3

    line = None
    if rank == 0:
        op_bytes = w.enc_bytes  # == rec_bytes for 2 erasures
        avg_op_ms = (enc_ms + rec_ms) / 2
        achieved = op_bytes / (avg_op_ms * 1e-3) / 1e9
        info = B.kernel_info(k, m, w.s)
        # each op is `disp` dispatches of the kernel, whole objects each
        tpo = -(-w.s // info["tile_bytes"])
        per_disp = max(1, vec_chunk_tiles() // tpo)
        disp = -(-n // per_disp)
        pmc, pmc_file, pmc_reject = load_pmc()
        traffic = traffic_disp = None
        if pmc and KERNEL_NAME in pmc.get("kernels", {}):
            traffic_disp = pmc["kernels"][KERNEL_NAME].get("hbm_bytes_per_launch")
            traffic = None if traffic_disp is None else traffic_disp * disp
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_steps": settle_steps,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: splitmix64 objects (SURVEY.md §8d), generated in HBM",
            "config": {
                "workload": "4+2 Encode + Reconstruct{0,1} of 4096 x 1 MiB objects per GPU, device-resident "
                            "(BASELINE configs[1]+[2])",
                "k": k, "m": m, "object_bytes": obj_len, "shard_bytes": w.s,
                "objects_per_gpu": n, "global_objects": n * world,
                "parallelism": f"object-partition x{world}",
                "bytes_per_step_per_gpu": step_bytes,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": KERNEL_NAME,
                "bytes_per_op": op_bytes,
                "dispatches_per_op": disp,
                "objects_per_dispatch": min(per_disp, n),
                "bytes_per_dispatch": op_bytes // disp,
                "traffic_per_dispatch": traffic_disp,
                "encode_ms_per_op": round(enc_ms, 4),
                "reconstruct_ms_per_op": round(rec_ms, 4),
                "ms_per_dispatch": round(avg_op_ms / disp, 4),
                "traffic_source": pmc_file if traffic is not None else None,
                "traffic_note": pmc_reject,
                "kernel_sources_sha256": kernel_sources_sha256(),
                "tile_bytes": info["tile_bytes"], "kernel_kind": info["kind"],
                "blocks_per_cu": info["blocks_per_cu"],
                # N > 1: each rank's own launches (the fields above use the max over ranks)
                "per_rank": None if per_rank is None else [
                    {"rank": r, "encode_ms_per_op": round(e, 4), "reconstruct_ms_per_op": round(c, 4),
                     "frac": round(op_bytes / ((e + c) / 2 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                    for r, (e, c) in enumerate(per_rank)],
            },
            "object_data_gib_s": round(value * k / (k + m), 2),
            "parity_ok": ok,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            ns = min(512, n)
            gpu = (w.objs[:ns].cpu().numpy(), w.parity[:ns].cpu().numpy(), w.rebuilt[:ns].cpu().numpy())
            line["cpu_baseline"] = cpu_baseline(k, m, obj_len, erased, budget_s=args.cpu_budget, sample_objs=ns,
                                                gpu=gpu if first == 0 else None)
            del gpu
    del w  # free this rank's headline batch before the partition / split buffers
    torch.cuda.empty_cache()
    if args.config5_objects > 0:
        c5 = config5(pg, k, m, obj_len, args.config5_objects, world, rank, ctl_device)
        if rank == 0:
            line["config5"] = c5
            ok = ok and c5.get("parity_ok", True)  # a skipped leg reports why, not a failure
    if rank == 0 and not args.no_small:
        try:
            line["small_objects"] = small_objects()
        except Exception as e:  # noqa: BLE001 - reported; never blocks the other ranks
            line["small_objects"] = {"error": f"{type(e).__name__}: {e}"[:200]}
        try:
            line["config4"] = config4()
        except Exception as e:  # noqa: BLE001 - reported; never blocks the other ranks
            line["config4"] = {"error": f"{type(e).__name__}: {e}"[:200]}
        try:
            line["odd_objects"] = odd_objects()
        except Exception as e:  # noqa: BLE001 - reported; never blocks the other ranks
            line["odd_objects"] = {"error": f"{type(e).__name__}: {e}"[:200]}
        try:
            line["random_objects"] = random_objects()
        except Exception as e:  # noqa: BLE001 - reported; never blocks the other ranks
            line["random_objects"] = {"error": f"{type(e).__name__}: {e}"[:200]}
        try:
            line["mid_objects"] = mid_objects()
        except Exception as e:  # noqa: BLE001 - reported; never blocks the other ranks
            line["mid_objects"] = {"error": f"{type(e).__name__}: {e}"[:200]}
    if world > 1 and backend == "nccl" and args.split_objects > 0:
        split = batch_split(pg, k, m, obj_len, args.split_objects, world, rank, ctl_device)
        if rank == 0:
            line["batch_split"] = split
            ok = ok and split.get("parity_ok", True)
    if not args.no_host_path:
        # rank 0 drives every GPU of the node from one process; the others wait
        if rank == 0:
            try:
                # its parity flag is reported in the object; the exit status
                # stays the headline's (and the split's)
                line["host_path"] = host_path(k, m, obj_len, all_devices=world > 1)
            except Exception as e:  # noqa: BLE001 - reported; never blocks the other ranks
                line["host_path"] = {"error": f"{type(e).__name__}: {e}"[:200]}
        if pg:
            pg.barrier()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if pg:
        pg.destroy_process_group()
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
