#!/usr/bin/env python3
"""Benchmark of the experiment-1 key/FK join (BASELINE.json metric) on the hj3d engine.

A "step" = one execution of the Csr plan (main_experiment1.cc:623-744): build the chaining
table on R.k, then probe it with every S tuple (unique-key early exit) and materialise the
output row-id pairs in HBM. Inputs are resident in HBM before timing.

Workloads (BASELINE.json configs):
  B  |R| = 1e7, |S| = 1e8 per GPU (the headline; default with --gpus 1; weak scaling with --gpus N)
  D  |R| = 1e8, |S| = 1e9 in total over N GPUs (default with --gpus N > 1; strong scaling): each
     rank holds a contiguous 1/N of both relations, bucket-range partitions them and exchanges the
     (key, row) pairs with one all-to-all per relation per step
  C  3D table on Zipf(0.8) S.a, Nrs plan (one GPU)
  E  experiment-4 deferred unnesting, Ndu plan (one GPU)
Inputs: --inputs reference (default) = the reference's own generator (hj3d_gen_exp1_ref /
hj3d_gen_exp4_ref, bit-exact with main_experiment1.cc:415-457 / main_experiment4.cc:517-575), so
the counters of the verification step are compared with the fixture the reference binary wrote
for exactly this workload (tests/golden/exp1_R<nR>_S<nS>_uni.json ...); --inputs device = seeded
device generators (verification by the key/FK pair identity).

value = probe tuples/s (all ranks' probe tuples / max over ranks of the probe-phase time, the
reference's t_probeStr); build_ms is reported beside it. ms_per_step = wall time per step.
"""
import argparse
import json
import os
import sys
import subprocess
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))

METRIC = "probe tuples/s + build ms, exp1 key/FK |R|=1e7 |S|=1e8, 1/2/4/8 GPU"
SEED_R, SEED_S = 0x5eed0001, 0x5eed0002
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_golden.out")
STAT_KEYS = ("nb", "empty", "entries", "distinct", "cc0_min", "cc0_max", "cc0_sum", "cc0_cnt",
             "cc1_min", "cc1_max", "cc1_sum", "cc1_cnt")
OUT_KEYS = ("n", "sum_a", "sum_b", "sum_h", "xor_h")


def lib_sha16():
    """sha256 (16 hex digits) of the libhj3d.so this process loads (HJ3D_LIB or the in-tree build)."""
    import hashlib
    path = os.environ.get("HJ3D_LIB") or os.path.join(ROOT, "3d-hashjoin_amd", "lib", "libhj3d.so")
    try:
        with open(path, "rb") as fh:
            return hashlib.sha256(fh.read()).hexdigest()[:16]
    except OSError:
        return None


def pmc_candidates(pattern):
    """PMC summaries under profiles/ matching `pattern`, best first: one taken on the library this
    process runs (its lib_sha16), then the most recently collected (collected_unix), then by name."""
    import glob
    me = lib_sha16()
    rows = []
    for path in glob.glob(os.path.join(ROOT, "profiles", pattern)):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        rows.append((d.get("lib_sha16") == me and me is not None, d.get("collected_unix", 0), path))
    return [p for _, _, p in sorted(rows, reverse=True)]


def latest_pmc():
    files = [p for p in pmc_candidates("r*_pmc.json") if not os.path.basename(p).split("_pmc")[0].endswith(
        ("_C", "_E", "_Dsh", "_D_shards"))]
    return files[0] if files else ""


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default=None, choices=["B", "C", "D", "E"],
                   help="B: headline key/FK chaining join, per GPU (default with --gpus 1); D: |R|=1e8 |S|=1e9 "
                        "in total over the GPUs (default with --gpus > 1); C: 3D table on Zipf(0.8) S.a, Nrs "
                        "plan; E: experiment-4 deferred unnesting (Ndu)")
    p.add_argument("--nR", type=int, default=None, help="|R| (B: per GPU, default 1e7; D: total, default 1e8)")
    p.add_argument("--nS", type=int, default=None, help="|S| (B: per GPU, default 1e8; D: total, default 1e9)")
    p.add_argument("--inputs", default="reference", choices=["reference", "device"],
                   help="reference: the reference's generator (bit-exact; counters checked against its fixture); "
                        "device: seeded device generators (checked by the key/FK pair identity)")
    p.add_argument("--b", type=int, default=1, help="bucket scale-down (#buckets = |R| / b)")
    p.add_argument("--no-emit", action="store_true", help="aggregate-only probe (no pair materialisation)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=20_000_000,
                   help="config B: the CPU baseline probes this prefix of the identical S relation")
    p.add_argument("--cpu-reps", type=int, default=8, help="CPU baseline: repeat_mintime minimum repetitions")
    p.add_argument("--no-mintime", action="store_true", help="skip the repeat_mintime figure")
    p.add_argument("--pmc-json", default=latest_pmc(), help="PMC summary (scripts/pmc_summary.py) for roofline.traffic")
    p.add_argument("--json-out", default=None)
    p.add_argument("--chunks", type=int, default=4,
                   help="N>1: S is exchanged in this many chunks, each chunk's all-to-all overlapping the "
                        "previous chunk's probe")
    p.add_argument("--dist-path", action="store_true",
                   help="N=1: run the multi-GPU strand (partition, RCCL exchange through libhj3d, bucket-range "
                        "table, chunked probe) on one GPU (the GPU test of that code path)")
    p.add_argument("--rehearse", action="store_true",
                   help="N>1 on ONE GPU: every rank on cuda:0, gloo exchange staged through host memory "
                        "(checks the multi-GPU code path; the numbers are not a scaling measurement)")
    p.add_argument("--xpart", default="single", choices=["single", "stable"],
                   help="N>1 probe side: single-pass exchange partitioner (hj3d_partition_strided) or the "
                        "stable two-pass one (hj3d_partition; A/B)")
    p.add_argument("--plan", default="Csr", choices=["Csr", "Nsr", "Nrs"],
                   help="workload B/D plan: Csr chaining build R / probe S (the headline); Nsr 3D table on R.k, "
                        "probe S + unnest; Nrs 3D table on S.a (NB = #dv(S.a) from the distributed pre-pass), "
                        "probe R + unnest")
    p.add_argument("--probe-path", default="packed", choices=["packed", "pairs"],
                   help="unique chaining probe: packed pairs, two launches (default), or the (hash, row) pair "
                        "partitioned probe (A/B)")
    p.add_argument("--theta", type=float, default=0.8, help="config C Zipf parameter")
    p.add_argument("--nested-build", default="agg", choices=["agg", "slices", "sort"],
                   help="3D build: bucket-range partition + LDS aggregation (default), the same on the packed "
                        "partitioner's slices (HJ3D_OPT_NESTED_PK, the form of tables above 2048 partitions), LSD "
                        "key sort (HJ3D_OPT_NESTED_SORT)")
    p.add_argument("--chain-build", default="auto", choices=["auto", "slices"],
                   help="chaining build: the library's choice (default), or the two-level slice build (pk_build, "
                        "HJ3D_OPT_PK_BUILD) wherever it applies (A/B)")
    p.add_argument("--torch-events", action="store_true",
                   help="phase boundaries timed with torch.cuda.Event (default hipEvents; A/B) instead of the "
                        "library's fence-free timing events")
    p.add_argument("--rp-unfused", action="store_true",
                   help="small build partitions as two launches (histogram, scatter) instead of the fused "
                        "one-launch partition (HJ3D_OPT_RP_UNFUSED, A/B)")
    p.add_argument("--lib-timing", default="auto", choices=["auto", "0", "1", "2"],
                   help="library timers (hj3d_ctx_timing): auto = 2 (dispatch-carried kernel spans only, no marker "
                        "packets between kernels) where the line's per-kernel figures come from those spans (the "
                        "packed probe), 1 (every timer) for the other B/D probe paths, 0 for C/E (no timer read)")
    p.add_argument("--log2R", type=int, default=22, help="config E: |R| = 2^log2R")
    a = p.parse_args()
    if a.workload is None:
        a.workload = "B" if a.gpus == 1 else "D"
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _host_cpu():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def fixture(name):
    """The reference's own counters for a workload (tests/golden, written by the reference binary)."""
    f = os.path.join(GOLDEN, name + ".json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        return json.load(fh)


def _run_ref(args, what):
    core = sorted(os.sched_getaffinity(0))[-1]
    p = subprocess.run([REF_BIN] + [str(a) for a in args], capture_output=True, text=True, timeout=900,
                       preexec_fn=lambda: os.sched_setaffinity(0, {core}))
    if p.returncode != 0:
        log(f"reference CPU baseline ({what}) failed (rc={p.returncode}): {p.stderr[-500:]}")
        return None
    return json.loads(p.stdout.strip().splitlines()[-1])


def cpu_baseline_reference(nR, nS, prefix, reps):
    """The reference's own Csr plan (main_experiment1.cc:636-699, compiled from /root/reference into
    oracle/_ref/ by oracle/Makefile) on the identical relations the GPU line joins (the reference
    generator at |R| = nR, |S| = nS), probing a bounded prefix of S; repeat_mintime (>= reps
    repetitions, >= 300 ms, clear_ht between), child process pinned to one core. None when the
    binary is absent (then the oracle port runs)."""
    if not os.path.exists(REF_BIN):
        return None
    r = _run_ref(["time_csr", nR, nS, reps, prefix], "Csr")
    if r is None:
        return None
    m = r["probe_prefix"]
    assert r["c_top"] == m, r  # every FK finds its key
    return {
        "value": m / (r["probe_ns"] * 1e-9),
        "unit": "probe tuples/s",
        "cores": 1,
        "kind": "reference",
        "sample": (f"the reference's Csr plan (AlgHashJoinBuild/AlgHashJoinProbe<unique>, HtChaining1) compiled from "
                   f"the reference sources (oracle/_ref/ref_golden.out time_csr) on the IDENTICAL relations of the GPU "
                   f"line (reference generator, mt19937 seed 5489, |R| = {nR}, |S| = {nS}): build all of R, probe the "
                   f"first {m} S tuples; repeat_mintime ({r['reps']} reps, >= 300 ms, clear_ht between), 1 pinned core"),
        "reps": r["reps"],
        "build_ms": r["build_ns"] * 1e-6,
        "probe_ms": r["probe_ns"] * 1e-6,
        "host_cpu": _host_cpu(),
        "nproc": os.cpu_count(),
    }


def cpu_baseline_reference_nrs(nR, nS, theta, reps):
    """Config C's CPU baseline: the reference's Nrs plan (3D table on Zipf S.a, probe R, unnest,
    counting Top; main_experiment1.cc:1001-1185) compiled from the reference sources
    (oracle/_ref/ref_golden.out time_nrs) on a bounded sample (|R|/10, |S|/10: one repetition on the
    full config C relation takes ~15 s on one core), repeat_mintime, one pinned core. Unit as the
    config C line: unnested output tuples per second of the probe strand."""
    if not os.path.exists(REF_BIN):
        return None
    r = _run_ref(["time_nrs", nR, nS, theta, reps], "Nrs")
    if r is None:
        return None
    assert r["c_unnest"] == nS, r  # every S tuple's key is in R
    return {
        "value": r["c_unnest"] / (r["probe_ns"] * 1e-9),
        "unit": "output tuples/s",
        "cores": 1,
        "kind": "reference",
        "sample": (f"the reference's Nrs plan (AlgNestJoinBuild on S.a, NB = #dv(S.a) = {r['nb']}; AlgNestJoinProbe "
                   f"-> AlgUnnestHt -> counting AlgTop) compiled from the reference sources "
                   f"(oracle/_ref/ref_golden.out time_nrs): |R| = {nR}, |S| = {nS} with S.a ~ Zipf({theta}) "
                   f"(reference generator, mt19937 seed 5489; a tenth of config C, since one repetition of the full "
                   f"workload takes ~15 s on one core), repeat_mintime ({r['reps']} reps), 1 pinned core"),
        "reps": r["reps"],
        "build_ms": r["build_ns"] * 1e-6,
        "probe_ms": r["probe_ns"] * 1e-6,
        "host_cpu": _host_cpu(),
        "nproc": os.cpu_count(),
    }


def cpu_baseline_reference_ndu(log2R, reps):
    """Config E's CPU baseline: the reference's Ndu plan (main_experiment4.cc:831-941: two 3D
    builds, R through both probes, deferred unnesting, counting Top) compiled from the reference
    sources (oracle/_ref/ref_golden.out time_ndu) on the identical workload of the GPU line (log2R,
    alpha=3 A=4 beta=2 B=2, the reference generator), repeat_mintime, one pinned core."""
    if not os.path.exists(REF_BIN):
        return None
    r = _run_ref(["time_ndu", log2R, 3, 4, 2, 2, reps], "Ndu")
    if r is None:
        return None
    return {
        "value": r["cardR"] / (r["probe_ns"] * 1e-9),
        "unit": "probe tuples/s",
        "cores": 1,
        "kind": "reference",
        "sample": (f"the reference's Ndu plan (two AlgNestJoinBuild, AlgScan(R) -> AlgNestJoinProbe(S) -> "
                   f"AlgNestJoinProbe(T) -> AlgUnnestHt x2 -> counting AlgTop) compiled from the reference sources "
                   f"(oracle/_ref/ref_golden.out time_ndu) on the identical config E relations (reference generator, "
                   f"log2R={log2R} alpha=3 A=4 beta=2 B=2, c_top = {r['c_top']}), repeat_mintime ({r['reps']} reps, "
                   f">= 300 ms, clear_ht between), 1 pinned core"),
        "reps": r["reps"],
        "build_ms": r["build_ns"] * 1e-6,
        "probe_ms": r["probe_ns"] * 1e-6,
        "host_cpu": _host_cpu(),
        "nproc": os.cpu_count(),
    }


def cpu_baseline_port(R_host, S_host, nb, reps):
    """The oracle's single-thread port of the reference Csr plan on a bounded sample, pinned
    to one core (reported baseline, not the target). Used when oracle/_ref is absent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # CPU baseline leg only

    out = {}

    def run():
        try:
            core = sorted(os.sched_getaffinity(0))[-1]
            os.sched_setaffinity(0, {core})  # this thread only
        except (AttributeError, OSError):
            pass
        out["res"] = O.chain_plan(R_host, 0, S_host, 1, nb, True, agg=False, min_ms=300.0, min_reps=reps)

    th = threading.Thread(target=run)
    th.start()
    th.join()
    r = out["res"]
    return {
        "value": len(S_host) / (r.probe_ns * 1e-9),
        "unit": "probe tuples/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"Csr plan of the oracle (oracle/hj3d_oracle.c, pointer-chained reference layout): build all "
                   f"{len(R_host)} R tuples, probe the first {len(S_host)} S tuples of the GPU line's relation, "
                   f"{r.reps} reps (repeat_mintime), 1 pinned core"),
        "build_ms": r.build_ns * 1e-6,
        "probe_ms": r.probe_ns * 1e-6,
        "host_cpu": _host_cpu(),
        "nproc": os.cpu_count(),
    }


def copy_peak(torch, ctx, dev, nbytes=1 << 30):
    """the streaming-copy peak measured in this run (hj3d_stream_copy on the engine's
    stream: 1 GiB read + 1 GiB written per launch, best of six variants x 5 launches), so the
    roofline fractions against 8 TB/s can be read against what this box actually streams."""
    try:
        src = torch.empty(nbytes // 4, dtype=torch.int32, device=dev).fill_(1)
        dst = torch.empty_like(src)
        r = ctx.stream_copy_peak(dst, src, 5)
        del src, dst
        return r
    except Exception as e:  # measurement only: the line still carries the 8 TB/s fractions
        log(f"copy peak not measured: {e}")
        return None


def _with_copy_peak(roof, cp, keys=("achieved",)):
    """Adds the same-run copy peak and the fractions of it to a roofline dict."""
    if not cp:
        roof["copy_peak_GBs"] = None
        return
    roof["copy_peak_GBs"] = cp["copy_peak_GBs"]
    roof["copy_peak"] = cp
    for k in keys:
        if roof.get(k):
            roof[f"{k}_frac_of_copy_peak" if k != "achieved" else "frac_of_copy_peak"] = roof[k] / cp["copy_peak_GBs"]


_EVENT_CTX = None  # the workload's hj3d context: phase events on its stream (hj3d.TimingEvent)


def _events(torch, n):
    """Phase-boundary events of one step. With a context: HIP events on the engine's stream created
    without the system-scope fence (hj3d_tevent_*): a default event writes the L2 back when it is
    recorded and leaves the GPU idle ~10 us at each phase boundary."""
    if _EVENT_CTX is not None:
        import hj3d
        return [hj3d.TimingEvent(_EVENT_CTX) for _ in range(n)]
    return [torch.cuda.Event(enable_timing=True) for _ in range(n)]


def _emit(line, args):
    s = json.dumps(line)
    print(s, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(s + "\n")


def main():
    args = parse()
    if args.workload in ("C", "E"):
        return main_single_config(args)
    import torch
    import hj3d

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    local = 0 if args.rehearse else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from hj3d import dist as hdist
    sharded = world > 1 or args.dist_path  # the partition + exchange strand
    if world > 1:
        import torch.distributed as dist
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    # ---- workload: global sizes and this rank's contiguous row ranges ----
    if args.workload == "B":  # per GPU, weak scaling
        nR_tot = (args.nR or 10_000_000) * world
        nS_tot = (args.nS or 100_000_000) * world
        scaling = "weak"
    else:  # D: in total, strong scaling
        nR_tot = args.nR or 100_000_000
        nS_tot = args.nS or 1_000_000_000
        scaling = "strong"
    r_lo, r_hi = rank * nR_tot // world, (rank + 1) * nR_tot // world
    s_lo, s_hi = rank * nS_tot // world, (rank + 1) * nS_tot // world
    nR, nS = r_hi - r_lo, s_hi - s_lo
    plan = args.plan
    emit = not args.no_emit
    ctx = hj3d.Context(local)
    global _EVENT_CTX
    _EVENT_CTX = None if args.torch_events else ctx
    # per-kernel HIP events: dispatch-carried spans (2) for the packed probe, every timer (1) otherwise.
    # With --lib-timing auto the K timed steps run uninstrumented (0) and K further steps carry the
    # kernel events (the line's per-kernel figures): an event riding on a dispatch costs ~10 us of
    # idle GPU before the next kernel (profiles/r05x_*), ~2 % of config B's probe phase.
    lib_timing = (2 if (args.probe_path == "packed" and args.plan == "Csr") else 1) if args.lib_timing == "auto" \
        else int(args.lib_timing)
    timed_timing = 0 if args.lib_timing == "auto" else lib_timing
    ctx.timing(timed_timing)
    if sharded and not args.rehearse:
        # the data path (counts, pairs, counter merges) on libhj3d's own RCCL communicator;
        # torch.distributed only hands over its id and times (barriers, max over ranks). World
        # size 1 (--dist-path): RCCL ships every chunk to this rank itself.
        hdist.use_comm(hdist.comm_from_torch(ctx) if world > 1 else hj3d.Comm(ctx, hj3d.Comm.unique_id(ctx), 0, 1))

    def teardown():
        # the library's communicator before torch's process group (both hold RCCL state)
        comm = hdist.current_comm()
        if comm is not None:
            torch.cuda.synchronize()
            comm.close()
            hdist.use_comm(None)
        if world > 1:
            torch.distributed.destroy_process_group()
    packed = args.probe_path == "packed" and plan == "Csr"
    ctx.packed_probe(packed)
    if args.nested_build == "slices":
        ctx.nested_pk(True)
    elif args.nested_build == "sort":
        ctx.nested_sort(True)
    if args.chain_build == "slices":
        ctx.pk_build(True)
    if args.rp_unfused:
        ctx.rp_unfused(True)
    fx = fixture(f"exp1_R{nR_tot}_S{nS_tot}_uni") if (args.inputs == "reference" and args.b == 1) else None
    fx_plan = (fx or {}).get("plans", {}).get(plan)

    # ---- inputs (HBM-resident before timing): rank r holds global rows [lo, hi) of R and S ----
    t_gen = time.perf_counter()
    R = torch.zeros((nR, 3), dtype=torch.int32, device=dev)
    S = torch.zeros((nS, 3), dtype=torch.int32, device=dev)
    Rk_full = None
    if args.inputs == "reference":
        # every rank runs the reference's sequential generator stream and keeps its slice
        if world > 1:  # generated once per node (local rank 0), memory-mapped by every rank
            maker = int(os.environ.get("LOCAL_RANK", "0")) == 0  # (--rehearse maps every rank to device 0)
            Rk_full, Sa = reference_columns_cached(nR_tot, nS_tot, maker, barrier)
        else:
            Rk_full, Sa = hj3d.gen_exp1_ref(nR_tot, nS_tot)
        R[:, 0] = torch.from_numpy(np.ascontiguousarray(Rk_full[r_lo:r_hi]).view("int32")).to(dev)
        S[:, 0] = torch.arange(s_lo, s_hi, dtype=torch.int64, device=dev).to(torch.int32)
        S[:, 1] = torch.from_numpy(np.ascontiguousarray(Sa[s_lo:s_hi]).view("int32")).to(dev)
        del Sa
        data = ("the reference's generator (hj3d_gen_exp1_ref = Experiment1::init, main_experiment1.cc:415-457, "
                "bit-exact: R.k = std::shuffle(iota), S.a ~ uniform_int over [0,|R|) then vec_permute, mt19937 seed 5489)")
    else:
        ctx.gen_keys(R, 0, r_lo, nR_tot, SEED_R)     # R.k: permutation of [0, |R|)
        ctx.gen_keys(S, 0, s_lo, 0, 0)               # S.k: global row id
        ctx.gen_fk(S, 1, s_lo, nR_tot, SEED_S)       # S.a ~ U[0, |R|)
        data = "synthetic (device-generated: R.k = seeded permutation of [0,|R|), S.a ~ U[0,|R|))"
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t_gen
    relR = hj3d.Rel(R, key_word=0, row_base=r_lo)
    relS = hj3d.Rel(S, key_word=1, row_base=s_lo)
    # plan: build side, probe side, table kind (main_experiment1.cc: Csr 623-848, Nrs 969-1076,
    # Nsr 1078-1185); every S tuple has exactly one partner, so each plan outputs |S| pairs
    if plan == "Nrs":
        # NB = #dv(S.a) / b: the pre-pass (bitmaps, all-to-all'ed slices, OR + popcount) outside
        # the timed region, as the reference counts numDvSa at generation time
        dv = hdist.num_distinct_rel(ctx, relS, nR_tot) if world > 1 else ctx.num_distinct(relS, nR_tot)
        nb = max(dv // args.b, 1)
        bT, pT, bRel, pRel, nB, nP, pkw, prow0 = S, R, relS, relR, nS, nR, 0, r_lo
    else:
        dv = None
        nb = max(nR_tot // args.b, 1)
        bT, pT, bRel, pRel, nB, nP, pkw, prow0 = R, S, relR, relS, nR, nS, 1, s_lo
    kind = hj3d.HJ3D_CHAIN if plan == "Csr" else hj3d.HJ3D_NESTED
    unique, unnest = plan == "Csr", plan != "Csr"

    C = max(1, args.chunks)
    if not sharded:
        table = hj3d.Table(ctx, kind, nb)
        table.reserve(nB)
        out = torch.empty((nS, 2), dtype=torch.int32, device=dev) if emit else None
    else:
        lo, hi = hj3d.part_range(nb, world, rank)
        table = hj3d.Table(ctx, kind, nb, lo, hi)
        sendB = torch.empty((nB, 2), dtype=torch.int32, device=dev)
        cntB = torch.zeros((1, world), dtype=torch.int64, device=dev)
        sb = [nP * c // C for c in range(C + 1)]
        pRel_c = [hj3d.Rel(pT[sb[c]:sb[c + 1]], key_word=pkw, row_base=prow0 + sb[c]) for c in range(C)]
        cntP = torch.zeros((C, world), dtype=torch.int64, device=dev)
        # probe side: the single-pass partitioner writes destination p of chunk c at rows
        # [p * stride_c, ...) of that chunk's send buffer (stride_c = the chunk's tuple count); the
        # build side keeps the stable two-pass partitioner (its order fixes long chains' order)
        single = args.xpart == "single"
        # stride_c = hj3d_partition_stride (mean + 8 sigma + 2 tiles per destination), so the send
        # buffer is ~ the chunk's pairs, not world x chunk; a chunk whose counts show a spill (a
        # destination above its stride: skewed keys) is re-partitioned by the stable partitioner
        # into `spill` and sent back to back (the counts are the same, so no rank notices)
        if single:
            xstride = [hj3d.partition_stride(sb[c + 1] - sb[c], world) for c in range(C)]
            sendP_c = [torch.empty((max(world * xstride[c], 1), 2), dtype=torch.int32, device=dev) for c in range(C)]
        else:
            xstride = [None] * C
            sendP = torch.empty((nP, 2), dtype=torch.int32, device=dev)
            sendP_c = [sendP[sb[c]:sb[c + 1]] for c in range(C)]
        spill = {}

        def part_probe(c):
            ctx.partition(pRel_c[c], nb, world, sendP_c[c], cntP[c], stride=xstride[c])

        def send_of(c, sc_c):
            """(send buffer, stride) of chunk c once its counts are known on the host."""
            if xstride[c] is None or max(sc_c) <= xstride[c]:
                return sendP_c[c], xstride[c]
            if c not in spill:
                spill[c] = torch.empty((max(sb[c + 1] - sb[c], 1), 2), dtype=torch.int32, device=dev)
            ctx.partition(pRel_c[c], nb, world, spill[c], cntP[c])
            return spill[c], None
        # receive buffers sized from the exchanged counts of a sizing pass (partition + counts
        # all-to-all): the inputs do not change between steps, so neither do the receive totals
        ctx.partition(bRel, nb, world, sendB, cntB[0])
        for c in range(C):
            part_probe(c)
        _, rcB = hdist.exchange_counts(cntB)
        _, rcP = hdist.exchange_counts(cntP)
        n_recvB, n_recvP = int(sum(rcB[0])), int(sum(sum(r) for r in rcP))
        table.reserve(max(n_recvB, 1))
        recvB = torch.empty((max(n_recvB, 1), 2), dtype=torch.int32, device=dev)
        recvP = torch.empty((max(n_recvP, 1), 2), dtype=torch.int32, device=dev)
        # key/FK: one output per S tuple; Csr / Nsr probe S (one dense slot per received probe
        # tuple), Nrs builds on S (its outputs are the received build tuples)
        n_out_cap = n_recvP if plan != "Nrs" else n_recvB
        out = torch.empty((max(n_out_cap, 1), 2), dtype=torch.int32, device=dev) if emit else None
    torch.cuda.synchronize()

    state = {}

    def step(ev):
        ev[0].record()
        if not sharded:
            table.build(bRel)
            ev[1].record()
            ctx.probe(table, pRel, unique=unique, unnest=unnest, out=out, fetch=False, checksum=state.get("ck", False))
        else:
            ctx.partition(bRel, nb, world, sendB, cntB[0])
            # with the receive capacity: every rank refuses together if any rank's buffer is short
            scB, rcB = hdist.exchange_counts(cntB, recv_cap=recvB.shape[0])
            rB, work = hdist.exchange_pairs_async(sendB, scB[0], rcB[0], recvB)
            if work is not None:
                work.wait()
            state["build_n"] = rB.shape[0]
            table.build(hj3d.Rel(rB, key_word=0, row_word=1))
            ev[1].record()
            # the probe side in C chunks: partition every chunk, exchange all chunks' counts in one
            # collective (one host synchronisation), start every chunk's pair all-to-all, then probe
            # chunk c as soon as its pairs have arrived (chunk c+1 in flight meanwhile); the chunks
            # accumulate into one probe strand
            for c in range(C):
                part_probe(c)
            scP, rcP = hdist.exchange_counts(cntP, recv_cap=recvP.shape[0])
            pend, roff = [], 0
            for c in range(C):
                sbuf, sstride = send_of(c, scP[c])
                rS, work = hdist.exchange_pairs_async(sbuf, scP[c], rcP[c], recvP[roff:], send_stride=sstride)
                roff += rS.shape[0]
                pend.append((rS, work))
            ooff = 0
            for c, (rS, work) in enumerate(pend):
                if work is not None:
                    work.wait()
                o = out[ooff:] if out is not None else None
                ctx.probe(table, hj3d.Rel(rS, key_word=0, row_word=1), unique=unique, unnest=unnest, out=o,
                          fetch=False, checksum=state.get("ck", False), accumulate=c > 0)
                # dense output (unique chaining): one slot per probe tuple; unnest: the count so far
                ooff = ooff + rS.shape[0] if unique else (ctx.probe_result().n_out if c + 1 < C else ooff)
            state["probe_n"] = roff
        ev[2].record()

    for _ in range(args.warmup):
        step(_events(torch, 3))
    torch.cuda.synchronize()
    barrier()
    ctx.timer_reset()
    evs = [_events(torch, 3) for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in evs:
        step(e)
    torch.cuda.synchronize()
    barrier()
    wall = time.perf_counter() - t0

    build_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    probe_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    instrumented = None
    if timed_timing != lib_timing:
        # K kernel-timing steps: the same step with the per-kernel events (HIP events on the engine's
        # stream, riding on the timed kernels' dispatches)
        ctx.timing(lib_timing)
        ctx.timer_reset()
        kevs = [_events(torch, 3) for _ in range(args.steps)]
        barrier()
        torch.cuda.synchronize()
        for e in kevs:
            step(e)
        torch.cuda.synchronize()
        barrier()
        instrumented = {"steps": args.steps, "lib_timing": lib_timing,
                        "build_ms": sum(e[0].elapsed_time(e[1]) for e in kevs) / args.steps,
                        "probe_ms": sum(e[1].elapsed_time(e[2]) for e in kevs) / args.steps}
    # per-kernel averages (HIP events on the engine's stream): over the timed steps, or over the
    # kernel-timing steps when the timed steps ran uninstrumented
    kern_avg = {}
    kprobe = "k_pk_probe" if packed else ("k_rp_probe_seg" if unique else "k_rn_probe_seg")
    kpart = "k_pk_part" if packed else "k_rp_part1"
    for name, ph in ((kprobe, hj3d.T_PROBE_KERNEL), (kpart, hj3d.T_SCATTER)) + \
            ((("k_pk_split", hj3d.T_HIST),) if packed else ()):
        ms, cnt = ctx.timer(ph)
        kern_avg[name] = ms / cnt if cnt else None
    ctx.timing(timed_timing)
    # verification step (outside the timed region): the same step once more with the
    # order-independent output checksums folded in
    state["ck"] = True
    step(_events(torch, 3))
    torch.cuda.synchronize()
    res = ctx.probe_result()
    st = table.stats()
    wall_ms = wall * 1e3 / args.steps
    probe_n_local = state.get("probe_n", nP)

    # repeat_mintime (util/measure_helpers.hh:15-41 as main_experiment1.cc:663-699 uses it): >= 8
    # repetitions, doubled while their total is below 300 ms, clear_ht between repetitions
    mintime = None
    if not sharded and not args.no_mintime:
        state["ck"] = False  # timed like the K steps: no verification checksums
        n_rep, tot_b, tot_p, i = 8, 0.0, 0.0, 0
        while i < n_rep:
            e = _events(torch, 3)
            step(e)
            torch.cuda.synchronize()
            tot_b += e[0].elapsed_time(e[1])
            tot_p += e[1].elapsed_time(e[2])
            if i == n_rep - 1 and tot_b + tot_p < 300.0:
                n_rep *= 2
            if i != n_rep - 1:
                table.clear()
            i += 1
        mintime = {"reps": n_rep, "total_ms": tot_b + tot_p, "build_ms": tot_b / n_rep, "probe_ms": tot_p / n_rep,
                   "value": nS / (tot_p / n_rep * 1e-3),
                   "protocol": "repeat_mintime(300 ms, min 8 reps), clear_ht between reps, hipEvents per phase"}

    # ---- verification of the verification step (bit-exact) ----
    got = {"n": res.n_out, "sum_a": res.sum_a, "sum_b": res.sum_b, "sum_h": res.sum_h, "xor_h": res.xor_h,
           "c_cmp": res.n_cmps, "c_matched": res.n_matched}
    if world > 1:
        s = hdist.allreduce_sum_u64([got[k] for k in ("n", "sum_a", "sum_b", "sum_h", "c_cmp", "c_matched")], dev)
        got.update(dict(zip(("n", "sum_a", "sum_b", "sum_h", "c_cmp", "c_matched"), s)))
        got["xor_h"] = hdist.allreduce_xor_u64(res.xor_h, dev)
        st = hdist.allreduce_stats(st, dev)
    verify = {}
    if fx_plan is not None:
        # the reference's own counters for exactly this workload (fixture written by the reference binary)
        ref_out = fx_plan["out"]
        verify["against"] = f"tests/golden/exp1_R{nR_tot}_S{nS_tot}_uni.json plan {plan} (reference binary)"
        verify["out"] = all(got[k] == ref_out[k] for k in OUT_KEYS)
        verify["c_htProbeCmp"] = got["c_cmp"] == fx_plan["c_cmp"]
        verify["c_top"] = (got["n"] if unnest or unique else got["c_matched"]) == fx_plan["c_top"]
        verify["stats"] = {k: st[k] for k in STAT_KEYS if k in fx_plan.get("stats", {})} == \
            {k: fx_plan["stats"][k] for k in STAT_KEYS if k in fx_plan.get("stats", {})}
    else:
        # the expected key/FK pair set without a hash table (inverse permutation of R.k)
        expd = torch.zeros(8, dtype=torch.int64, device=dev)
        if args.inputs == "device":
            ctx.expected_fk_join_gen(relS, nR_tot, SEED_R, swap=plan == "Nrs", res=expd)
        else:
            Rfull = torch.zeros((nR_tot, 3), dtype=torch.int32, device=dev)
            Rfull[:, 0] = torch.from_numpy(Rk_full.view("int32")).to(dev)
            e = ctx.expected_fk_join(hj3d.Rel(Rfull, 0), relS, nR_tot, swap=plan == "Nrs")
            expd[:5] = torch.tensor([e[k] - (1 << 64) if e[k] >= (1 << 63) else e[k] for k in OUT_KEYS])
            del Rfull
        torch.cuda.synchronize()
        exp_local = [int(x) & hj3d.MASK64 for x in expd.cpu().tolist()[:5]]
        if world > 1:
            exp_local = hdist.allreduce_sum_u64(exp_local[:4], dev) + [hdist.allreduce_xor_u64(exp_local[4], dev)]
        verify["against"] = "expected key/FK pair set (inverse permutation of R.k, no hash table)"
        verify["out"] = [got[k] for k in OUT_KEYS] == exp_local
    verify["c_top_is_S"] = got["n"] == nS_tot
    verified = all(v for k, v in verify.items() if k != "against")

    if world > 1:
        build_ms = hdist.allreduce_max(build_ms, dev)
        probe_ms_local = probe_ms
        probe_ms = hdist.allreduce_max(probe_ms, dev)
        wall_ms = hdist.allreduce_max(wall_ms, dev)
        kern_avg = {k: (hdist.allreduce_max(v, dev) if v is not None else None) for k, v in kern_avg.items()}
        # per-GPU imbalance of the bucket-range partition (a Zipf hot key's bucket
        # lands on one GPU): received tuples and phase times, min / max over ranks
        loc = {"build_tuples": float(state.get("build_n", nB)), "probe_tuples": float(probe_n_local),
               "probe_ms": float(probe_ms_local)}
        per_gpu = {}
        for k, v in loc.items():
            mx, mn = hdist.allreduce_max(v, dev), -hdist.allreduce_max(-v, dev)
            sm = hdist.allreduce_sum_u64([int(round(v * 1000))], dev)[0] / 1000.0
            per_gpu[k] = {"min": mn, "max": mx, "max_over_mean": mx / (sm / world) if sm else None}

    if rank != 0:
        teardown()
        if not verified:
            raise SystemExit(f"rank {rank}: verification failed")
        return

    # ---- roofline of the dominant kernel ----
    # Algorithmic bytes per launch, n = probe tuples of this rank per launch:
    #   k_pk_part (k_rp_part1)      n * (12 + 8)   read the S tuple (AoS {k,a,b}), write the packed pair
    #   k_pk_split (tables of more than 1024 LDS slices: the second partition level)
    #                               n * (8 + 8)    read the coarse pair, write the fine pair
    #   k_pk_probe (k_rp_probe_seg) n * (8 + 8) + |R| * 8 + nb * 4   read the pair, write the output pair, stage
    #                                                    the table slices (entries + directory) once
    #   k_rn_probe_seg  (3D plans, unnest materialised): n * (8 + 16) read the pair, write the slot's
    #                   output count (8), sub offset and probe row (4 + 4); + the slices (directory +
    #                   16-B main records) once. The expansion kernels that follow are not in this timer.
    # (N > 1: the probe side is the received pair array, 8 B per tuple.)
    launches = C if sharded else 1
    n = probe_n_local / launches
    tuple_bytes = 8 if sharded else 12
    if unique:
        alg = {kpart: n * (tuple_bytes + 8), "k_pk_split": n * 16,
               kprobe: n * (8 + (8 if emit else 0)) + (nR_tot // world) * 8 + (nb // world) * 4}
    else:
        n_keys = dv if plan == "Nrs" else nR_tot
        alg = {kpart: n * (tuple_bytes + 8),
               kprobe: n * (8 + (16 if emit else 0)) + (n_keys // world) * 16 + (nb // world) * 4}
    kernels = {}
    for k, ms in kern_avg.items():
        if ms:
            kernels[k] = {"avg_ms": ms, "alg_bytes": alg[k], "achieved_GBs": alg[k] / (ms * 1e-3) / 1e9,
                          "frac": alg[k] / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS}
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
    traffic, pmc = None, None
    if not sharded and plan == "Csr" and args.pmc_json and os.path.exists(args.pmc_json):
        try:
            with open(args.pmc_json) as f:
                pm = json.load(f)
            if pm.get("workload", "B") == "B" and pm.get("nS") == nS and pm.get("nR") == nR and pm.get("emit") == emit:
                pmc = pm.get("kernels", {})
                traffic = (pmc.get(dom) or {}).get("traffic_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    pmc_src = os.path.relpath(args.pmc_json, ROOT) if pmc else None
    if pmc:
        for k in kernels:
            if k in pmc:
                kernels[k]["traffic"] = pmc[k].get("traffic_bytes_per_launch")
    # the whole probe phase (partition + probe; N > 1: + exchange) against SURVEY §8(d): 20 B per
    # probe tuple + per output 8 B (chaining) or 4 + 8 B (unnest: sub row read, pair write)
    phase_alg = probe_n_local * (tuple_bytes + 8) + (nS_tot // world) * ((8 if emit else 0) + (0 if unique else 4))
    if unique:
        metric, unit = METRIC, "probe tuples/s"
    else:
        metric, unit = (f"unnested output tuples/s (probe + unnest phase), exp1 key/FK plan {plan}",
                        "output tuples/s")
    if args.workload == "B":
        workload = f"exp1 key/FK plan {plan}, |R|={nR_tot // world} |S|={nS_tot // world} per GPU, uniform FKs, b={args.b}"
    else:
        workload = (f"config D: exp1 key/FK plan {plan}, |R|={nR_tot} |S|={nS_tot} in total over {world} GPU(s) "
                    f"(|R|={nR} |S|={nS} on rank 0), uniform FKs, b={args.b}")

    # The roofline's unit. Unique chaining (Csr): the longer of the two timed probe-phase kernels, which
    # are the step's largest. The 3D plans: the step's largest kernels are the build's aggregation
    # (k_nagg) and the unnest expansion (k_expand_light), which carry no per-kernel timers, so the line
    # is bounded on the probe + unnest PHASE (SURVEY §8(d) bytes) and reports the build phase beside it;
    # the timed partition / probe kernels stay under roofline.kernels.
    if unique:
        roof = {"bound": "hbm", "achieved": kernels[dom]["achieved_GBs"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": kernels[dom]["frac"], "traffic": traffic, "kernel": dom,
                "kernel_avg_ms": kernels[dom]["avg_ms"], "alg_bytes_per_launch": kernels[dom]["alg_bytes"]}
    else:
        # build: read the 12-B tuple, write the (hash, row) pair, read it back, write the 4-B sub row
        build_alg = (nB if sharded else (nS_tot if plan.startswith("Nrs") else nR_tot) // world) * (12 + 8 + 8 + 4)
        roof = {"bound": "hbm", "achieved": phase_alg / (probe_ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": phase_alg / (probe_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, "traffic": None,
                "kernel": "phase (probe + unnest)", "alg_bytes_per_launch": phase_alg,
                "note": "3D plan: the step's largest kernels (k_nagg in the build, k_expand_light in the unnest) "
                        "have no per-kernel timers; the line is bounded on the probe + unnest phase",
                "build_phase": {"ms": build_ms, "alg_bytes": build_alg,
                                "achieved_GBs": build_alg / (build_ms * 1e-3) / 1e9,
                                "frac": build_alg / (build_ms * 1e-3) / 1e9 / PEAK_HBM_GBS}}
    line = {
        "metric": metric,
        "value": nS_tot / (probe_ms * 1e-3),  # |S| probe tuples (Csr) = |S| output pairs (every plan)
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall_ms,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": data,
        "config": {
            "workload": workload, "config": args.workload,
            "plan": plan, "R_total": nR_tot, "S_total": nS_tot, "R_per_gpu": nR_tot // world,
            "S_per_gpu": nS_tot // world, "num_buckets": nb, "num_dv_Sa": dv,
            "emit_pairs": emit, "parallelism": f"bucket-range partition x{world}" if sharded else "single GPU",
            "exchange_chunks": (C if sharded else None),
            "exchange_partitioner": ((("single-pass hj3d_partition_strided" if args.xpart == "single" else
                                       "stable two-pass hj3d_partition") + " (probe side); stable (build side)")
                                     if sharded else None),
            "exchange": ("libhj3d hj3d_comm_* over RCCL" if sharded and not args.rehearse else
                         "torch.distributed gloo, host-staged (rehearsal)" if sharded else None),
            "rehearsal_one_gpu": bool(args.rehearse),
            # the packed probe's LDS-slice geometry on this rank: P slices of W buckets; C > 1 = two
            # partition levels (k_pk_part into P1 ranges of C slices, k_pk_split by slice)
            "probe_slices": ctx.pk_plan(max(nb // world, 1), max(nB, 1)) if packed else None,
        },
        "build_ms": build_ms,
        "probe_ms": probe_ms,
        "join_tuples_per_s": nS_tot / ((build_ms + probe_ms) * 1e-3),
        "input_generation_s": gen_s,
        "roofline": {
            **roof,
            "kernels": kernels,
            "kernel_timing": ("HIP events riding on the kernels' dispatches over K kernel-timing steps after the "
                              "(uninstrumented) timed steps" if instrumented else
                              "HIP events on the engine's stream over the timed steps"),
            "instrumented_steps": instrumented,
            "probe_phase": {"ms": probe_ms, "alg_bytes": phase_alg,
                            "achieved_GBs": phase_alg / (probe_ms * 1e-3) / 1e9,
                            "frac": phase_alg / (probe_ms * 1e-3) / 1e9 / PEAK_HBM_GBS},
        },
        "repeat_mintime": mintime,
        "counters": {"c_top": got["n"], "c_htProbeCmp": got["c_cmp"],
                     "reference_c_htProbeCmp": fx_plan["c_cmp"] if fx_plan else None,
                     "stats": {k: st[k] for k in STAT_KEYS}},
        "verification": verify,
        "verified_bit_exact": verified,
    }
    if pmc_src:
        line["roofline"]["pmc_source"] = pmc_src
        line["roofline"]["pmc_same_library"] = pm.get("lib_sha16") is not None and pm.get("lib_sha16") == lib_sha16()
    _with_copy_peak(line["roofline"], copy_peak(torch, ctx, dev))
    pp = line["roofline"]["probe_phase"]
    if line["roofline"].get("copy_peak_GBs"):
        pp["frac_of_copy_peak"] = pp["achieved_GBs"] / line["roofline"]["copy_peak_GBs"]
    if world > 1:
        line["per_gpu"] = per_gpu
    if sharded:
        line["config"]["probe_send_pairs"] = sum(int(t.shape[0]) for t in sendP_c) if single else nP
        line["config"]["probe_spilled_chunks"] = sorted(spill)
    line["cpu_baseline"] = None
    if world == 1 and not args.no_cpu_baseline and plan == "Csr":
        m = min(args.cpu_sample, nS)
        if args.inputs == "reference":
            line["cpu_baseline"] = cpu_baseline_reference(nR, nS, m, args.cpu_reps)
        if line["cpu_baseline"] is None:
            R_host = R.cpu().numpy().view("uint32")
            S_host = S[:m].cpu().numpy().view("uint32")
            line["cpu_baseline"] = cpu_baseline_port(R_host, S_host, nb, args.cpu_reps)
    _emit(line, args)
    teardown()
    if not verified:
        raise SystemExit(f"verification failed: {verify}")


def reference_columns_cached(nR, nS, maker, barrier):
    """The reference's experiment-1 columns (R.k, S.a) for N > 1 ranks: the generator is one
    sequential mt19937 stream (minutes of one core at config D), so one process per node
    (`maker`) runs it and writes relation files under $HJ3D_REL_CACHE (default
    $TMPDIR/hj3d_relcache), reused by later runs; every rank then maps them and copies its slice."""
    import tempfile
    from hj3d import relfile
    d = os.environ.get("HJ3D_REL_CACHE", os.path.join(tempfile.gettempdir(), "hj3d_relcache"))
    meta = {"gen": "hj3d_gen_exp1_ref", "nR": nR, "nS": nS, "skew": 0, "theta": 1.0, "t": 0}
    pr, ps = os.path.join(d, f"exp1_R{nR}_S{nS}_Rk.rel"), os.path.join(d, f"exp1_R{nR}_S{nS}_Sa.rel")

    def valid(p):
        try:
            return relfile.read_header(p).get("meta") == meta
        except (OSError, ValueError):
            return False

    import hj3d
    if maker and not (valid(pr) and valid(ps)):
        try:
            os.makedirs(d, exist_ok=True)
            Rk, Sa = hj3d.gen_exp1_ref(nR, nS)
            relfile.save(pr, Rk.reshape(-1, 1), 0, meta)
            relfile.save(ps, Sa.reshape(-1, 1), 0, meta)
            del Rk, Sa
        except OSError as e:  # no room for the cache: every rank generates for itself below
            print(f"relation cache under {d} not written ({e})", file=sys.stderr)
            for f in (pr, ps, pr + ".tmp", ps + ".tmp"):
                try:
                    os.remove(f)
                except OSError:
                    pass
    barrier()
    if not (valid(pr) and valid(ps)):
        return hj3d.gen_exp1_ref(nR, nS)
    return relfile.load(pr, verify=False)[0][:, 0], relfile.load(ps, verify=False)[0][:, 0]


def _load_pmc(path, workload):
    """The PMC summary at `path` if it was taken on `workload` (scripts/pmc_summary.py)."""
    cands = ([path] if path else []) + pmc_candidates(f"r*_{workload}_pmc.json")
    pm = None
    for path in cands:
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload", "B") == workload:
            pm = d
            break
    if pm is None:
        return None
    pm["_path"] = os.path.relpath(path, os.path.dirname(os.path.abspath(__file__)))
    pm["_same_library"] = pm.get("lib_sha16") is not None and pm.get("lib_sha16") == lib_sha16()
    return pm


def main_single_config(args):
    """Configs C and E of BASELINE.json (one GPU). Same protocol as config B: the reference's own
    inputs generated and resident before timing, W warmup steps, K timed steps bracketed by
    synchronize, one verification step after timing whose counters are compared with the fixture
    the reference binary wrote for exactly this workload."""
    import torch
    import hj3d

    if int(os.environ.get("WORLD_SIZE", "1")) != 1 or args.gpus != 1:
        raise SystemExit("--workload C/E run on one GPU")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ctx = hj3d.Context(0)
    global _EVENT_CTX
    _EVENT_CTX = None if args.torch_events else ctx
    launches = []  # (build, probe) kernel launches of each step
    ctx.timing(0 if args.lib_timing == "auto" else int(args.lib_timing))  # (no timer is read here)
    if args.rp_unfused:
        ctx.rp_unfused(True)
    if args.nested_build == "sort":
        ctx.nested_sort(True)
    elif args.nested_build == "slices":
        ctx.nested_pk(True)

    if args.workload == "C":
        nR, nS = args.nR or 10_000_000, args.nS or 100_000_000
        R, S = hj3d.exp1_relations_ref(nR, nS, True, args.theta, 0, device=dev)
        relR, relS = hj3d.Rel(R, key_word=0), hj3d.Rel(S, key_word=1)
        dv = ctx.num_distinct(relS, nR)  # NB = #dv(S.a) as the reference sizes Nrs (main_experiment1.cc:1001)
        table = hj3d.Table(ctx, hj3d.HJ3D_NESTED, dv)
        table.reserve(nS)
        out = torch.empty((nS, 2), dtype=torch.int32, device=dev)
        state = {"ck": False}
        fx = fixture(f"exp1_R{nR}_S{nS}_zipf{str(args.theta).replace('.', '').rstrip('0') or '0'}")

        def step(ev):
            l0 = hj3d.lib().hj3d_launch_count()
            ev[0].record()
            table.build(relS)
            ev[1].record()
            l1 = hj3d.lib().hj3d_launch_count()
            ctx.probe(table, relR, unnest=True, out=out, fetch=False, checksum=state["ck"])
            ev[2].record()
            launches.append((l1 - l0, hj3d.lib().hj3d_launch_count() - l1))

    else:
        log2R, a, A, b, B = args.log2R, 3, 4, 2, 2
        nR = 1 << log2R
        R, S, T = hj3d.exp4_relations_ref(log2R, a, A, b, B, device=dev)
        nb = (nR >> a) + (nR >> b)  # numFkCommon + numFkExclusive (main_experiment4.cc:855)
        ts, tt = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb), hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb)
        ts.reserve(S.shape[0])
        tt.reserve(T.shape[0])
        relR, relS, relT = hj3d.Rel(R, key_word=0), hj3d.Rel(S, key_word=1), hj3d.Rel(T, key_word=1)
        fx = fixture(f"exp4_R{log2R}_a{a}_A{A}_b{b}_B{B}")
        state = {"ck": False}

        def step(ev):
            l0 = hj3d.lib().hj3d_launch_count()
            ev[0].record()
            ctx.build_many([ts, tt], [relS, relT])  # one launch sequence for both tables
            ev[1].record()
            l1 = hj3d.lib().hj3d_launch_count()
            # (the triple hashes only in the verification step, as the other workloads' checksums)
            ctx.probe2(ts, tt, relR, fetch=False, checksum=state["ck"])
            ev[2].record()
            launches.append((l1 - l0, hj3d.lib().hj3d_launch_count() - l1))

    torch.cuda.synchronize()
    for _ in range(args.warmup):
        step(_events(torch, 3))
    torch.cuda.synchronize()
    evs = [_events(torch, 3) for _ in range(args.steps)]
    del launches[:]  # the timed steps' kernel launches (build, probe), from the library's own counter
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in evs:
        step(e)
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t0) * 1e3 / args.steps
    build_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    probe_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    timed_launches = launches[-1] if launches else (None, None)

    verify = {}
    if args.workload == "C":
        state["ck"] = True
        step(_events(torch, 3))
        torch.cuda.synchronize()
        r = ctx.probe_result()
        got = {"n": r.n_out, "sum_a": r.sum_a, "sum_b": r.sum_b, "sum_h": r.sum_h, "xor_h": r.xor_h}
        counters = {"c_htProbe": r.n_matched, "c_htProbeCmp": r.n_cmps, "c_unnest": r.n_out, "numDvSa": dv}
        if fx is not None:
            ref = fx["plans"]["Nrs"]
            verify["against"] = f"tests/golden/exp1_R{nR}_S{nS}_zipf08.json plan Nrs (reference binary)"
            verify["numDvSa"] = dv == fx["numDvSa"]
            verify["counters"] = (r.n_matched, r.n_cmps, r.n_out) == (ref["c_probe"], ref["c_cmp"], ref["c_unnest"])
            verify["out"] = all(got[k] == ref["out"][k] for k in OUT_KEYS)
            st = table.stats()
            verify["stats"] = all(st[k] == ref["stats"][k] for k in STAT_KEYS)
        else:
            exp = ctx.expected_fk_join(relR, relS, nR, swap=True)
            verify["against"] = "expected key/FK pair set"
            verify["out"] = got == exp and r.n_out == nS
        n_out = r.n_out
        # phase bytes: build 20 B/tuple; probe 20 B/probe + unnest 12 B/output
        build_bytes, probe_bytes = nS * 20, nR * 20 + n_out * 12
        workload = (f"config C: exp1 plan Nrs (3D table on S.a, probe R, unnest), |R|={nR} |S|={nS}, "
                    f"S.a ~ Zipf({args.theta})")
        data = ("the reference's generator (hj3d_gen_exp1_ref = Experiment1::init with zipf_distribution, "
                f"theta={args.theta}, bit-exact)")
        metric, unit, value = ("unnested output tuples/s (probe + unnest phase), config C", "output tuples/s",
                               n_out / (probe_ms * 1e-3))
        n_build = nS
    else:
        state["ck"] = True  # verification step: the same step with the triple checksums folded in
        step(_events(torch, 3))
        torch.cuda.synchronize()
        r = ctx.probe2_result()
        counters = {k: r[k] for k in ("c_probe_rs", "c_probe_rs_cmp", "c_probe_rt", "c_probe_rt_cmp", "c_unnest_1",
                                      "c_unnest_2", "c_top")}
        if fx is not None:
            ref = fx["plans"]["Ndu"]
            verify["against"] = f"tests/golden/exp4_R{log2R}_a3_A4_b2_B2.json plan Ndu (reference binary)"
            verify["counters"] = all(counters[k] == ref[k2] for k, k2 in (
                ("c_probe_rs", "c_probe_RS"), ("c_probe_rs_cmp", "c_probe_RS_cmp"), ("c_probe_rt", "c_probe_RT"),
                ("c_probe_rt_cmp", "c_probe_RT_cmp"), ("c_unnest_1", "c_unnest_1"), ("c_unnest_2", "c_unnest_2"),
                ("c_top", "c_top")))
            if "out" in ref:
                verify["out"] = all(r[k] == ref["out"][k] for k in ("sum_a", "sum_b", "sum_c", "sum_h", "xor_h"))
        else:
            nc, A = nR >> 3, 4
            verify["against"] = "analytic counters of experiment 4"
            verify["counters"] = (r["c_top"] == nc * A * A and r["c_unnest_1"] == nc * A and r["c_probe_rt"] == nc
                                  and r["c_probe_rs"] == nc + (nR >> 2))
        n_out = r["c_top"]
        n_build = S.shape[0] + T.shape[0]
        build_bytes = n_build * 16  # 8-B {k,a} tuple read + 8 B (key,row) written
        probe_bytes = nR * 8 * 2 + n_out * 12
        workload = (f"config E: exp4 plan Ndu (two 3D probes, deferred unnesting), log2R={log2R} alpha=3 A=4 beta=2 "
                    f"B=2, |S|=|T|={S.shape[0]}")
        data = "the reference's generator (hj3d_gen_exp4_ref = Experiment4::init, bit-exact)"
        metric, unit, value = ("probe tuples/s (R through both 3D probes + deferred unnest), config E",
                               "probe tuples/s", nR / (probe_ms * 1e-3))
    verified = all(v for k, v in verify.items() if k != "against")
    line = {
        "metric": metric, "value": value, "unit": unit, "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall_ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": data, "config": {"workload": workload, "config": args.workload, "parallelism": "single GPU"},
        "build_ms": build_ms, "probe_ms": probe_ms,
        "launches_per_step": {"build": timed_launches[0], "probe": timed_launches[1],
                              "note": "kernel launches of libhj3d per timed step (hj3d_launch_count)"},
        "roofline": {"bound": "hbm", "kernel": "phase (build / probe)", "unit": "GB/s", "peak": PEAK_HBM_GBS,
                     "achieved": probe_bytes / (probe_ms * 1e-3) / 1e9,
                     "frac": probe_bytes / (probe_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, "traffic": None,
                     "build_achieved": build_bytes / (build_ms * 1e-3) / 1e9},
        "counters": counters, "verification": verify, "verified_bit_exact": verified, "cpu_baseline": None,
    }
    # HBM traffic of the phases from a PMC summary of this workload (scripts/gpu_pmc.sh +
    # scripts/pmc_summary.py --workload C|E): bytes per step of each phase's kernels
    pm = _load_pmc(args.pmc_json, args.workload)
    if pm:
        ph_build = ("k_rp_hist", "k_rp_scatter", "k_rp_wscatter", "k_rp_fused", "k_nagg", "k_nagg_mains", "k_rs_scatter",
                    "k_rs_hist")
        ph_probe = ("k_rp_part1", "k_rn_probe_seg", "k_expand_light", "k_expand_heavy_flat", "k_ndu_seg", "k_ndu",
                    "k_ndu_heavy")
        tr = {k: d.get("traffic_bytes_per_launch") for k, d in pm["kernels"].items()
              if d.get("traffic_bytes_per_launch")}
        line["roofline"]["traffic"] = sum(v for k, v in tr.items() if k in ph_probe) or None
        line["roofline"]["build_traffic"] = sum(v for k, v in tr.items() if k in ph_build) or None
        line["roofline"]["build_alg_bytes"] = build_bytes
        line["roofline"]["probe_alg_bytes"] = probe_bytes
        line["roofline"]["kernel_traffic"] = {
            k: {"traffic": v, "fetch": pm["kernels"][k].get("fetch_bytes"), "write": pm["kernels"][k].get("write_bytes")}
            for k, v in tr.items() if k in ph_build + ph_probe}
        line["roofline"]["pmc_source"] = pm.get("_path")
        line["roofline"]["pmc_same_library"] = pm.get("_same_library")
    _with_copy_peak(line["roofline"], copy_peak(torch, ctx, dev), keys=("achieved", "build_achieved"))
    if args.workload == "C" and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_reference_nrs(max(nR // 10, 1), max(nS // 10, 1), args.theta,
                                                          args.cpu_reps)
    elif args.workload == "E" and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_reference_ndu(log2R, args.cpu_reps)
    _emit(line, args)
    if not verified:
        raise SystemExit(f"verification failed: {verify}")


if __name__ == "__main__":
    main()
