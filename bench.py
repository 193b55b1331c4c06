#!/usr/bin/env python3
"""Benchmark of the experiment-1 key/FK join (BASELINE.json metric) on the hj3d engine.

A "step" = one execution of the Csr plan (main_experiment1.cc:623-744): build the chaining
table on R.k, then probe it with every S tuple (unique-key early exit) and materialise the
output row-id pairs in HBM. Inputs are resident in HBM before timing. Per GPU:
|R| = 1e7, |S| = 1e8 (BASELINE config B); with --gpus N (one process per GPU, torchrun) the
relations are N times larger and bucket-range partitioned with an RCCL all-to-all per step
(weak scaling).

value = probe tuples/s (all ranks' probe tuples / max over ranks of the probe-phase time, the
reference's t_probeStr); build_ms is reported beside it. ms_per_step = build + probe.
"""
import argparse
import json
import os
import sys
import subprocess
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))

METRIC = "probe tuples/s + build ms, exp1 key/FK |R|=1e7 |S|=1e8, 1/2/4/8 GPU"
SEED_R, SEED_S = 0x5eed0001, 0x5eed0002
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def latest_pmc():
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")))
    return files[-1] if files else ""


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--nR", type=int, default=10_000_000, help="|R| per GPU")
    p.add_argument("--nS", type=int, default=100_000_000, help="|S| per GPU")
    p.add_argument("--b", type=int, default=1, help="bucket scale-down (#buckets = |R| / b)")
    p.add_argument("--no-emit", action="store_true", help="aggregate-only probe (no pair materialisation)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=20_000_000, help="S tuples probed by the CPU baseline")
    p.add_argument("--cpu-reps", type=int, default=3)
    p.add_argument("--pmc-json", default=latest_pmc(), help="PMC summary (scripts/pmc_summary.py) for roofline.traffic")
    p.add_argument("--json-out", default=None)
    p.add_argument("--chunks", type=int, default=4,
                   help="N>1: S is exchanged in this many chunks, each chunk's all-to-all overlapping the "
                        "previous chunk's probe")
    p.add_argument("--rehearse", action="store_true",
                   help="N>1 on ONE GPU: every rank on cuda:0, gloo exchange staged through host memory "
                        "(checks the multi-GPU code path; the numbers are not a scaling measurement)")
    p.add_argument("--plan", default="Csr", choices=["Csr", "Nsr", "Nrs"],
                   help="workload B plan: Csr chaining build R / probe S (the headline); Nsr 3D table on R.k, "
                        "probe S + unnest; Nrs 3D table on S.a (NB = #dv(S.a) from the distributed pre-pass), "
                        "probe R + unnest (config D's per-GPU 3D join)")
    p.add_argument("--workload", default="B", choices=["B", "C", "E"],
                   help="B: the headline key/FK chaining join (default); C: 3D table on Zipf(0.8) S.a, Nrs plan; "
                        "E: experiment-4 deferred unnesting (Ndu)")
    p.add_argument("--theta", type=float, default=0.8, help="config C Zipf parameter")
    p.add_argument("--nested-build", default="agg", choices=["agg", "sort", "radix"],
                   help="3D build: bucket-range partition + LDS aggregation (default), LSD key sort "
                        "(HJ3D_OPT_NESTED_SORT), radix bucket CSR + per-bucket grouping (HJ3D_OPT_NESTED_RADIX)")
    p.add_argument("--log2R", type=int, default=23, help="config E: |R| = 2^log2R")
    return p.parse_args()


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


REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_golden.out")


def cpu_baseline_reference(nR, nS, reps):
    """The reference's own Csr plan (main_experiment1.cc:636-699, compiled from /root/reference
    into oracle/_ref/ by oracle/Makefile) on a bounded uniform key/FK sample, run as a child
    process pinned to one core. None when the binary is absent (then the oracle port runs)."""
    if not os.path.exists(REF_BIN):
        return None
    core = sorted(os.sched_getaffinity(0))[-1]
    p = subprocess.run([REF_BIN, "time_csr", str(nR), str(nS), str(reps)], capture_output=True, text=True,
                       timeout=600, preexec_fn=lambda: os.sched_setaffinity(0, {core}))
    if p.returncode != 0:
        log(f"reference CPU baseline failed (rc={p.returncode}): {p.stderr[-500:]}")
        return None
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["c_top"] == nS, r  # every FK finds its key
    return {
        "value": nS / (r["probe_ns"] * 1e-9),
        "unit": "probe tuples/s",
        "cores": 1,
        "kind": "reference",
        "sample": (f"the reference's Csr plan (AlgHashJoinBuild/AlgHashJoinProbe<unique>, HtChaining1) "
                   f"compiled from the reference sources (oracle/_ref/ref_golden.out time_csr): build {nR} R "
                   f"tuples, probe {nS} uniform-FK S tuples (reference generator, mt19937 seed 5489), "
                   f"{reps} reps, clear_ht between reps, 1 pinned core"),
        "build_ms": r["build_ns"] * 1e-6,
        "probe_ms": r["probe_ns"] * 1e-6,
        "host_cpu": _host_cpu(),
        "nproc": os.cpu_count(),
    }


def cpu_baseline_reference_nrs(nR, nS, theta, reps):
    """Config C's CPU baseline: the reference's Nrs plan (3D table on Zipf S.a, probe R, unnest,
    counting Top; main_experiment1.cc:1001-1185) compiled from the reference sources
    (oracle/_ref/ref_golden.out time_nrs) on a bounded sample (|R|/10, |S|/10), one pinned core.
    Unit as the config C line: unnested output tuples per second of the probe strand."""
    if not os.path.exists(REF_BIN):
        return None
    core = sorted(os.sched_getaffinity(0))[-1]
    p = subprocess.run([REF_BIN, "time_nrs", str(nR), str(nS), str(theta), str(reps)], capture_output=True,
                       text=True, timeout=600, preexec_fn=lambda: os.sched_setaffinity(0, {core}))
    if p.returncode != 0:
        log(f"reference CPU baseline (Nrs) failed (rc={p.returncode}): {p.stderr[-500:]}")
        return None
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["c_unnest"] == nS, r  # every S tuple's key is in R
    return {
        "value": r["c_unnest"] / (r["probe_ns"] * 1e-9),
        "unit": "output tuples/s",
        "cores": 1,
        "kind": "reference",
        "sample": (f"the reference's Nrs plan (AlgNestJoinBuild on S.a, NB = #dv(S.a) = {r['nb']}; AlgNestJoinProbe "
                   f"-> AlgUnnestHt -> counting AlgTop) compiled from the reference sources "
                   f"(oracle/_ref/ref_golden.out time_nrs): |R| = {nR}, |S| = {nS} with S.a ~ Zipf({theta}) "
                   f"(reference generator, mt19937 seed 5489), {reps} reps, clear_ht between reps, 1 pinned core"),
        "build_ms": r["build_ns"] * 1e-6,
        "probe_ms": r["probe_ns"] * 1e-6,
        "host_cpu": _host_cpu(),
        "nproc": os.cpu_count(),
    }


def cpu_baseline_reference_ndu(log2R, reps):
    """Config E's CPU baseline: the reference's Ndu plan (main_experiment4.cc:831-941: two 3D
    builds, R through both probes, deferred unnesting, counting Top) compiled from the reference
    sources (oracle/_ref/ref_golden.out time_ndu) on the same workload as the GPU line (log2R,
    alpha=3 A=4 beta=2 B=2, the reference generator), one pinned core."""
    if not os.path.exists(REF_BIN):
        return None
    core = sorted(os.sched_getaffinity(0))[-1]
    p = subprocess.run([REF_BIN, "time_ndu", str(log2R), "3", "4", "2", "2", str(reps)], capture_output=True,
                       text=True, timeout=600, preexec_fn=lambda: os.sched_setaffinity(0, {core}))
    if p.returncode != 0:
        log(f"reference CPU baseline (Ndu) failed (rc={p.returncode}): {p.stderr[-500:]}")
        return None
    r = json.loads(p.stdout.strip().splitlines()[-1])
    return {
        "value": r["cardR"] / (r["probe_ns"] * 1e-9),
        "unit": "probe tuples/s",
        "cores": 1,
        "kind": "reference",
        "sample": (f"the reference's Ndu plan (two AlgNestJoinBuild, AlgScan(R) -> AlgNestJoinProbe(S) -> "
                   f"AlgNestJoinProbe(T) -> AlgUnnestHt x2 -> counting AlgTop) compiled from the reference sources "
                   f"(oracle/_ref/ref_golden.out time_ndu): the full config E workload, log2R={log2R} alpha=3 A=4 "
                   f"beta=2 B=2 (c_top = {r['c_top']}), {reps} reps, clear_ht between reps, 1 pinned core"),
        "build_ms": r["build_ns"] * 1e-6,
        "probe_ms": r["probe_ns"] * 1e-6,
        "host_cpu": _host_cpu(),
        "nproc": os.cpu_count(),
    }


def cpu_baseline(R_host, S_host, nb, reps):
    """The oracle's single-thread port of the reference Csr plan on a bounded sample, pinned
    to one core (reported baseline, not the target). Used when oracle/_ref is absent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # CPU baseline leg only

    out = {}

    def run():
        try:
            core = sorted(os.sched_getaffinity(0))[-1]
            os.sched_setaffinity(0, {core})  # this thread only
            out["core"] = core
        except (AttributeError, OSError):
            pass
        out["res"] = O.chain_plan(R_host, 0, S_host, 1, nb, True, agg=False, min_ms=0.0, min_reps=reps)

    th = threading.Thread(target=run)
    th.start()
    th.join()
    r = out["res"]
    cpu_model = _host_cpu()
    return {
        "value": len(S_host) / (r.probe_ns * 1e-9),
        "unit": "probe tuples/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"Csr plan of the oracle (oracle/hj3d_oracle.c, pointer-chained reference layout): build all "
                   f"{len(R_host)} R tuples, probe the first {len(S_host)} S tuples, {r.reps} reps, 1 pinned core"),
        "build_ms": r.build_ns * 1e-6,
        "probe_ms": r.probe_ns * 1e-6,
        "host_cpu": cpu_model,
        "nproc": os.cpu_count(),
    }


def main():
    args = parse()
    if args.workload != "B":
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
    if world > 1:
        import torch.distributed as dist
        from hj3d import dist as hdist
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    nR, nS = args.nR, args.nS
    nR_tot = nR * world
    plan = args.plan
    emit = not args.no_emit
    ctx = hj3d.Context(local)
    ctx.timing(True)

    # ---- inputs (HBM-resident before timing): rank r holds global rows [r*n, (r+1)*n) ----
    R = torch.zeros((nR, 3), dtype=torch.int32, device=dev)
    S = torch.zeros((nS, 3), dtype=torch.int32, device=dev)
    ctx.gen_keys(R, 0, rank * nR, nR_tot, SEED_R)     # R.k: permutation of [0, |R|)
    ctx.gen_keys(S, 0, rank * nS, 0, 0)               # S.k: global row id
    ctx.gen_fk(S, 1, rank * nS, nR_tot, SEED_S)       # S.a ~ U[0, |R|)
    relR = hj3d.Rel(R, key_word=0, row_base=rank * nR)
    relS = hj3d.Rel(S, key_word=1, row_base=rank * nS)
    # plan: build side, probe side, table kind (main_experiment1.cc: Csr 623-848, Nrs 969-1076,
    # Nsr 1078-1185); every S tuple has exactly one partner, so each plan outputs |S| pairs
    if plan == "Nrs":
        # NB = #dv(S.a) / b: the pre-pass (bitmaps, all-to-all'ed slices, OR + popcount) outside
        # the timed region, as the reference counts numDvSa at generation time
        dv = hdist.num_distinct_rel(ctx, relS, nR_tot) if world > 1 else ctx.num_distinct(relS, nR_tot)
        nb = max(dv // args.b, 1)
        bT, pT, bRel, pRel, nB, nP, pkw, prow0 = S, R, relS, relR, nS, nR, 0, rank * nR
    else:
        dv = None
        nb = max(nR_tot // args.b, 1)
        bT, pT, bRel, pRel, nB, nP, pkw, prow0 = R, S, relR, relS, nR, nS, 1, rank * nS
    kind = hj3d.HJ3D_CHAIN if plan == "Csr" else hj3d.HJ3D_NESTED
    unique, unnest = plan == "Csr", plan != "Csr"
    n_out_local = nS  # output pairs of this rank's share (uniform FKs: |S| per rank)

    if world == 1:
        table = hj3d.Table(ctx, kind, nb)
        table.reserve(nB)
        out = torch.empty((n_out_local, 2), dtype=torch.int32, device=dev) if emit else None
    else:
        lo, hi = hj3d.part_range(nb, world, rank)
        table = hj3d.Table(ctx, kind, nb, lo, hi)
        slack = 1.05
        table.reserve(int(nB * slack) + 4096)
        sendB = torch.empty((nB, 2), dtype=torch.int32, device=dev)
        sendP = torch.empty((nP, 2), dtype=torch.int32, device=dev)
        cntB = torch.zeros(world, dtype=torch.int64, device=dev)
        C = max(1, args.chunks)
        sb = [nP * c // C for c in range(C + 1)]
        pRel_c = [hj3d.Rel(pT[sb[c]:sb[c + 1]], key_word=pkw, row_base=prow0 + sb[c]) for c in range(C)]
        cntP = torch.zeros((C, world), dtype=torch.int64, device=dev)
        recvB = torch.empty((int(nB * slack) + 4096, 2), dtype=torch.int32, device=dev)
        recvP = torch.empty((int(nP * slack) + 4096, 2), dtype=torch.int32, device=dev)
        out = torch.empty((int(n_out_local * slack) + 4096, 2), dtype=torch.int32, device=dev) if emit else None
    torch.cuda.synchronize()

    state = {}

    def probe_chunk(pend, ooff, first):
        rS, work = pend
        if work is not None:
            work.wait()
        n = rS.shape[0]
        o = out[ooff:] if out is not None else None
        ctx.probe(table, hj3d.Rel(rS, key_word=0, row_word=1), unique=unique, unnest=unnest, out=o, fetch=False,
                  checksum=state.get("ck", False), accumulate=not first)
        # outputs of this chunk: one per probe tuple (unique chaining probe, dense slots), else the
        # unnest count so far (read back: the next chunk's slots follow)
        return ooff + n if unique else ctx.probe_result().n_out

    def step(ev):
        ev[0].record()
        if world == 1:
            table.build(bRel)
            ev[1].record()
            ctx.probe(table, pRel, unique=unique, unnest=unnest, out=out, fetch=False, checksum=state.get("ck", False))
        else:
            ctx.partition(bRel, nb, world, sendB, cntB)
            rB = hdist.exchange(sendB, cntB, recvB)
            state["build_n"] = rB.shape[0]
            table.build(hj3d.Rel(rB, key_word=0, row_word=1))
            ev[1].record()
            # the probe side in C chunks: partition chunk c, start its all-to-all, then probe
            # chunk c-1 while chunk c is in flight (results accumulate into one probe strand)
            roff, ooff, pend, first = 0, 0, None, True
            for c in range(C):
                ctx.partition(pRel_c[c], nb, world, sendP[sb[c]:sb[c + 1]], cntP[c])
                rS, work = hdist.exchange_async(sendP[sb[c]:sb[c + 1]], cntP[c], recvP[roff:])
                roff += rS.shape[0]
                if pend is not None:
                    ooff = probe_chunk(pend, ooff, first)
                    first = False
                pend = (rS, work)
            ooff = probe_chunk(pend, ooff, first)
            state["probe_n"] = roff
        ev[2].record()

    def events():
        return [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    for _ in range(args.warmup):
        step(events())
    torch.cuda.synchronize()
    barrier()
    ctx.timer_reset()
    evs = [events() for _ in range(args.steps)]
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
    # per-kernel averages over the timed steps (HIP events on the engine's stream)
    kern_avg = {}
    kprobe = "k_rp_probe_seg" if unique else "k_rn_probe_seg"
    for name, ph in ((kprobe, hj3d.T_PROBE_KERNEL), ("k_rp_part1", hj3d.T_SCATTER)):
        ms, cnt = ctx.timer(ph)
        kern_avg[name] = ms / cnt if cnt else None
    # verification step (outside the timed region): the same step once more with the
    # order-independent output checksums folded in, compared below with the expected pair set
    state["ck"] = True
    step(events())
    torch.cuda.synchronize()
    res = ctx.probe_result()
    wall_ms = wall * 1e3 / args.steps
    probe_n_local = state.get("probe_n", nP)

    # ---- verification of the last step (bit-exact, size-independent) ----
    expd = torch.zeros(8, dtype=torch.int64, device=dev)
    ctx.expected_fk_join_gen(relS, nR_tot, SEED_R, swap=plan == "Nrs", res=expd)
    torch.cuda.synchronize()
    exp_local = [int(x) & hj3d.MASK64 for x in expd.cpu().tolist()[:5]]
    got_local = [res.n_out, res.sum_a, res.sum_b, res.sum_h]
    if world > 1:
        exp_sum = hdist.allreduce_sum_u64(exp_local[:4], dev)
        exp_xor = hdist.allreduce_xor_u64(exp_local[4], dev)
        got_sum = hdist.allreduce_sum_u64(got_local, dev)
        got_xor = hdist.allreduce_xor_u64(res.xor_h, dev)
        cmps = hdist.allreduce_sum_u64([res.n_cmps], dev)[0]
        build_ms = hdist.allreduce_max(build_ms, dev)
        probe_ms = hdist.allreduce_max(probe_ms, dev)
        wall_ms = hdist.allreduce_max(wall_ms, dev)
        kern_avg = {k: (hdist.allreduce_max(v, dev) if v is not None else None) for k, v in kern_avg.items()}
        # per-GPU imbalance of the bucket-range partition (a Zipf hot key's bucket
        # lands on one GPU): received tuples and phase times, min / max over ranks
        local = {"build_tuples": float(state.get("build_n", nB)), "probe_tuples": float(probe_n_local),
                 "probe_ms": float(sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps)}
        per_gpu = {}
        for k, v in local.items():
            mx, mn = hdist.allreduce_max(v, dev), -hdist.allreduce_max(-v, dev)
            sm = hdist.allreduce_sum_u64([int(round(v * 1000))], dev)[0] / 1000.0
            per_gpu[k] = {"min": mn, "max": mx, "max_over_mean": mx / (sm / world) if sm else None}
    else:
        exp_sum, exp_xor = exp_local[:4], exp_local[4]
        got_sum, got_xor = got_local, res.xor_h
        cmps = res.n_cmps
    verified = exp_sum == got_sum and exp_xor == got_xor and got_sum[0] == nS * world

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    # ---- roofline of the dominant kernel ----
    # Algorithmic bytes per launch (DESIGN.md "Kernels"), n = probe tuples of this rank:
    #   k_rp_part1      n * (12 + 8)                read the S tuple (AoS {k,a,b}), write the (hash,row) pair
    #   k_rp_probe_seg  n * (8 + 8) + |R| * 8 + nb * 4   read the pair, write the output pair, stage
    #                                                    the table slices (entries + directory) once
    # (N > 1: the probe side is the received pair array, 8 B per tuple.)
    launches = 1 if world == 1 else max(1, args.chunks)
    n = probe_n_local / launches  # probe tuples per kernel launch
    tuple_bytes = 12 if world == 1 else 8
    #   k_rn_probe_seg (3D plans, unnest materialised): n * (8 + 16) read the pair, write the slot's
    #                  output count (8), sub offset and probe row (4 + 4); + the slices (directory +
    #                  16-B main records) once. The expansion kernels that follow are not in this timer.
    if unique:
        alg = {
            "k_rp_part1": n * (tuple_bytes + 8),
            kprobe: n * (8 + (8 if emit else 0)) + (nR_tot // world) * 8 + (nb // world) * 4,
        }
    else:
        n_keys = dv if plan == "Nrs" else nR_tot
        alg = {
            "k_rp_part1": n * (tuple_bytes + 8),
            kprobe: n * (8 + (16 if emit else 0)) + (n_keys // world) * 16 + (nb // world) * 4,
        }
    kernels = {}
    for k, ms in kern_avg.items():
        if ms:
            kernels[k] = {"avg_ms": ms, "alg_bytes": alg[k], "achieved_GBs": alg[k] / (ms * 1e-3) / 1e9,
                          "frac": alg[k] / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS}
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
    traffic = None
    pmc = None
    if world == 1 and plan == "Csr" and args.pmc_json and os.path.exists(args.pmc_json):
        try:
            with open(args.pmc_json) as f:
                pm = json.load(f)
            if pm.get("nS") == nS and pm.get("nR") == nR and pm.get("emit") == emit:
                pmc = pm.get("kernels", {})
                traffic = (pmc.get(dom) or {}).get("traffic_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    if pmc:
        for k in kernels:
            if k in pmc:
                kernels[k]["traffic"] = pmc[k].get("traffic_bytes_per_launch")
    # the whole probe phase (partition + probe; N > 1: + exchange) against SURVEY §8(d): 20 B per
    # probe tuple + per output 8 B (chaining) or 4 + 8 B (unnest: sub row read, pair write)
    phase_alg = probe_n_local * (tuple_bytes + 8) + nS * ((8 if emit else 0) + (0 if unique else 4))
    if unique:
        metric, unit = METRIC, "probe tuples/s"
    else:
        metric, unit = (f"unnested output tuples/s (probe + unnest phase), exp1 key/FK plan {plan}",
                        "output tuples/s")

    line = {
        "metric": metric,
        "value": nS * world / (probe_ms * 1e-3),  # |S| probe tuples (Csr) = |S| output pairs (every plan)
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (device-generated: R.k = seeded permutation of [0,|R|), S.a ~ U[0,|R|))",
        "config": {
            "workload": f"exp1 key/FK plan {plan}, |R|={nR} |S|={nS} per GPU, uniform FKs, b={args.b}",
            "plan": plan, "R_per_gpu": nR, "S_per_gpu": nS, "num_buckets": nb, "num_dv_Sa": dv,
            "emit_pairs": emit, "parallelism": f"bucket-range partition x{world}" if world > 1 else "single GPU",
            "exchange_chunks": (max(1, args.chunks) if world > 1 else None),
            "rehearsal_one_gpu": bool(args.rehearse),
        },
        "build_ms": build_ms,
        "probe_ms": probe_ms,
        "join_tuples_per_s": nS * world / ((build_ms + probe_ms) * 1e-3),
        "roofline": {
            "bound": "hbm", "achieved": kernels[dom]["achieved_GBs"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": kernels[dom]["frac"], "traffic": traffic,
            "kernel": dom, "kernel_avg_ms": kernels[dom]["avg_ms"], "alg_bytes_per_launch": kernels[dom]["alg_bytes"],
            "kernels": kernels,
            "probe_phase": {"ms": probe_ms, "alg_bytes": phase_alg,
                            "achieved_GBs": phase_alg / (probe_ms * 1e-3) / 1e9,
                            "frac": phase_alg / (probe_ms * 1e-3) / 1e9 / PEAK_HBM_GBS},
        },
        "counters": {"c_top": got_sum[0], "c_htProbeCmp": cmps},
        "verified_bit_exact": verified,
    }
    if world > 1:
        line["per_gpu"] = per_gpu
    if world == 1 and not args.no_cpu_baseline and plan == "Csr":
        m = min(args.cpu_sample, nS)
        line["cpu_baseline"] = cpu_baseline_reference(nR, m, args.cpu_reps)
        if line["cpu_baseline"] is None:
            R_host = R.cpu().numpy().view("uint32")
            S_host = S[:m].cpu().numpy().view("uint32")
            line["cpu_baseline"] = cpu_baseline(R_host, S_host, nb, args.cpu_reps)
    else:
        line["cpu_baseline"] = None
    s = json.dumps(line)
    print(s, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(s + "\n")
    if world > 1:
        torch.distributed.destroy_process_group()
    if not verified:
        raise SystemExit("verification failed: join output differs from the expected key/FK pair set")


def _events(torch, n):
    return [torch.cuda.Event(enable_timing=True) for _ in range(n)]


def _emit(line, args):
    s = json.dumps(line)
    print(s, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(s + "\n")


def main_single_config(args):
    """Configs C and E of BASELINE.json (one GPU). Same protocol as config B: inputs generated and
    resident before timing, W warmup steps, K timed steps bracketed by synchronize, one
    verification step after timing (bit-exact identities)."""
    import torch
    import hj3d

    if int(os.environ.get("WORLD_SIZE", "1")) != 1 or args.gpus != 1:
        raise SystemExit("--workload C/E run on one GPU")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ctx = hj3d.Context(0)
    ctx.timing(True)
    if args.nested_build == "radix":
        ctx.nested_radix(True)
    elif args.nested_build == "sort":
        ctx.nested_sort(True)

    if args.workload == "C":
        nR, nS = args.nR, args.nS
        R = torch.zeros((nR, 3), dtype=torch.int32, device=dev)
        S = torch.zeros((nS, 3), dtype=torch.int32, device=dev)
        ctx.gen_keys(R, 0, 0, nR, SEED_R)
        ctx.gen_keys(S, 0, 0, 0, 0)
        ctx.gen_zipf(S, 1, 0, nR, args.theta, SEED_S)
        relR, relS = hj3d.Rel(R, key_word=0), hj3d.Rel(S, key_word=1)
        probe_t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nR)
        probe_t.build(relS)
        dv = probe_t.stats()["distinct"]  # NB = #dv(S.a) as the reference sizes Nrs (main_experiment1.cc:1001)
        del probe_t
        table = hj3d.Table(ctx, hj3d.HJ3D_NESTED, dv)
        table.reserve(nS)
        out = torch.empty((nS, 2), dtype=torch.int32, device=dev)
        state = {"ck": False}

        def step(ev):
            ev[0].record()
            table.build(relS)
            ev[1].record()
            ctx.probe(table, relR, unnest=True, out=out, fetch=False, checksum=state["ck"])
            ev[2].record()

        n_probe, n_build = nR, nS
    else:
        import numpy as np
        log2R, a, A, b, B = args.log2R, 3, 4, 2, 2
        nR = 1 << log2R
        nc, ne = nR >> a, nR >> b
        rng = np.random.default_rng(5489)
        common = np.repeat(np.arange(nc, dtype=np.uint32), A)
        exS = np.repeat(np.arange(nc, nc + ne, dtype=np.uint32), B)
        exT = np.repeat(np.arange(nc + ne, nc + 2 * ne, dtype=np.uint32), B)
        Sa = np.concatenate([rng.permutation(common), rng.permutation(exS)])
        Ta = np.concatenate([rng.permutation(common), rng.permutation(exT)])

        def rel2(a_col):
            t = np.zeros((len(a_col), 2), dtype=np.uint32)
            t[:, 0] = np.arange(len(a_col), dtype=np.uint32)
            t[:, 1] = a_col
            return torch.from_numpy(t.view(np.int32)).to(dev)

        R = rel2(np.zeros(nR, dtype=np.uint32))
        S, T = rel2(Sa), rel2(Ta)
        nb = nc + ne  # numFkCommon + numFkExclusive (main_experiment4.cc:855)
        ts, tt = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb), hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb)
        ts.reserve(len(Sa))
        tt.reserve(len(Ta))
        relR, relS, relT = hj3d.Rel(R, key_word=0), hj3d.Rel(S, key_word=1), hj3d.Rel(T, key_word=1)
        state = {}

        def step(ev):
            ev[0].record()
            ts.build(relS)
            tt.build(relT)
            ev[1].record()
            ctx.probe2(ts, tt, relR, fetch=False)
            ev[2].record()

        n_probe, n_build = nR, len(Sa) + len(Ta)

    torch.cuda.synchronize()
    for _ in range(args.warmup):
        step(_events(torch, 3))
    torch.cuda.synchronize()
    evs = [_events(torch, 3) for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in evs:
        step(e)
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t0) * 1e3 / args.steps
    build_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    probe_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps

    if args.workload == "C":
        state["ck"] = True
        step(_events(torch, 3))
        torch.cuda.synchronize()
        r = ctx.probe_result()
        exp = ctx.expected_fk_join(relR, relS, nR, swap=True)
        got = {"n": r.n_out, "sum_a": r.sum_a, "sum_b": r.sum_b, "sum_h": r.sum_h, "xor_h": r.xor_h}
        verified = got == exp and r.n_out == nS and r.n_matched == dv
        n_out = r.n_out
        counters = {"c_htProbe": r.n_matched, "c_htProbeCmp": r.n_cmps, "c_unnest": r.n_out, "numDvSa": dv}
        # phase bytes: build 20 B/tuple; probe 20 B/probe + unnest 12 B/output
        build_bytes, probe_bytes = nS * 20, nR * 20 + n_out * 12
        workload = f"exp1 plan Nrs (3D table on S.a, probe R, unnest), |R|={nR} |S|={nS}, S.a ~ Zipf({args.theta})"
        data = f"synthetic (device-generated: R.k = seeded permutation, S.a ~ Zipf(theta={args.theta}) over [0,|R|))"
        metric, unit, value = ("unnested output tuples/s (probe + unnest phase), config C", "output tuples/s",
                               n_out / (probe_ms * 1e-3))
    else:
        r = ctx.probe2_result()
        nc, A = nR >> 3, 4
        verified = (r["c_top"] == nc * A * A and r["c_unnest_1"] == nc * A and r["c_probe_rt"] == nc
                    and r["c_probe_rs"] == nc + (nR >> 2))
        counters = {k: r[k] for k in ("c_probe_rs", "c_probe_rs_cmp", "c_probe_rt", "c_probe_rt_cmp", "c_unnest_1",
                                      "c_unnest_2", "c_top")}
        n_out = r["c_top"]
        build_bytes = n_build * 16  # 8-B {k,a} tuple read + 8 B (key,row) written
        probe_bytes = nR * 8 * 2 + n_out * 12
        workload = (f"exp4 plan Ndu (two 3D probes, deferred unnesting), log2R={args.log2R} alpha=3 A=4 beta=2 B=2, "
                    f"|S|=|T|={len(Sa)}")
        data = "synthetic (numpy: R.k = iota, S.a/T.a = shuffled FK blocks as main_experiment4.cc:517-575)"
        metric, unit, value = ("probe tuples/s (R through both 3D probes + deferred unnest), config E",
                               "probe tuples/s", nR / (probe_ms * 1e-3))
    line = {
        "metric": metric, "value": value, "unit": unit, "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall_ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": data, "config": {"workload": workload, "parallelism": "single GPU"},
        "build_ms": build_ms, "probe_ms": probe_ms,
        "roofline": {"bound": "hbm", "kernel": "phase (build / probe)", "unit": "GB/s", "peak": PEAK_HBM_GBS,
                     "achieved": probe_bytes / (probe_ms * 1e-3) / 1e9,
                     "frac": probe_bytes / (probe_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, "traffic": None,
                     "build_achieved": build_bytes / (build_ms * 1e-3) / 1e9},
        "counters": counters, "verified_bit_exact": verified, "cpu_baseline": None,
    }
    if args.workload == "C" and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_reference_nrs(max(nR // 10, 1), max(nS // 10, 1), args.theta,
                                                          args.cpu_reps)
    elif args.workload == "E" and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_reference_ndu(args.log2R, args.cpu_reps)
    _emit(line, args)
    if not verified:
        raise SystemExit("verification failed")


if __name__ == "__main__":
    main()
