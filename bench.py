"""bench.py — RB-PHD-SLAM filter steps/s on MI355X (BASELINE.json metric).

A step = one pass of the hot path over one batch: Ackerman/CV predict + the
fused static GM-PHD (config 3: GM-CPHD) update (in-range split, EKF, births, weights, prune,
merge) + log-weight normalisation + nEff + (device-decided) stratified
resample.  Replay mode, like the reference's profile_run (main.cpp:1314-1321):
a fixed prior of exactly N x G components and a fixed measurement set, so
every step does identical work; the prior stays resident in HBM.

    python bench.py                      # N=1, config 3: 4096 x 512 x 64, CV + CPHD
    python bench.py --config 2           # 1024 x 256 x 32, Ackerman + PHD
    python bench.py --config 1           # the CPU oracle alone over the reference's data (configs[0])
    torchrun --nproc-per-node N bench.py --gpus N   # weak scaling, particles sharded

The default workload is the north-star's named target shape (BASELINE.json:
"≥10k filter update steps/s at 4096 particles × 512 GM components × 64
measurements on 1 MI355X, ≥6× at 8 GPUs") = configs[2] (config 3).  At N GPUs
every GPU steps a config-3-sized shard (4096 particles) of ONE filter whose
resample is global (RCCL all-gather + minimal migration): at N=8 that is the
32768 x 512 x 64 job of configs[3] (config 4), so value(8)/value(1) is the
north-star's c4 ÷ c3 scaling ratio.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def algorithmic_bytes(sizes_in, sizes_out, M):
    """B_step = Σ_n (28 G_in + 28 G_out + 32) + 12 M."""
    import numpy as np
    return int(28 * np.sum(sizes_in, dtype=np.int64) + 28 * np.sum(sizes_out, dtype=np.int64)
               + 32 * len(sizes_in) + 12 * M)


def _oracle_rate(config_id, n, threads, budget_s, phd_only=False, births=False):
    """Particle-updates/s of the optimised oracle build (oracle/liboracle_fast.so:
    predict [+ the scan's births, as the GPU step] + update + normalize) on a
    bounded sample of the config's workload (n = the particles per GPU the bench
    line ran), the sample's particles spread over `threads` OpenMP threads."""
    import phdslam
    import pyoracle
    cfg, _, G, M, df = phdslam.preset(config_id)
    ns = min(n, max(16, 4 * threads))
    c, poses, lw, maps, offs, z = phdslam.config_scenario(config_id, n=ns)
    if phd_only:
        c.filterType = 0
    cv = c.motionType != 1  # config 3: constant-velocity predict (phdfilter.cu:827-859)
    noise = pyoracle.noise_cv(c, ns, 1, 1) if cv else pyoracle.noise_ackerman(c, ns, 1, 1)
    used = pyoracle.set_threads(threads, fast=True)
    reps = 0
    t0 = time.perf_counter()
    while True:
        p2 = (pyoracle.predict_cv(c, poses, noise, fast=True) if cv
              else pyoracle.predict_ackerman(c, poses, 2.0, 0.05, noise, fast=True))
        m2, o2 = pyoracle.add_births(c, p2, maps, offs, z, fast=True) if births else (maps, offs)
        _, _, delta, _ = pyoracle.update(c, p2, m2, o2, z, fast=True)
        pyoracle.normalize(lw + delta, fast=True)
        reps += 1
        dt = time.perf_counter() - t0
        if dt > budget_s:
            break
    return reps * ns / dt, reps, ns, n, G, M, dt, used


def _ranges(cpus):
    cpus = sorted(cpus)
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(f"{cpus[i]}-{cpus[j]}" if j > i else str(cpus[i]))
        i = j + 1
    return ",".join(out)


def cpu_baseline(config_id, n, budget_s=12.0, births=False):
    """The oracle (same C++ source as the checker, built -O3 -march=x86-64-v3
    with OpenMP over particles: oracle/liboracle_fast.so) on a bounded sample of
    the same workload, 1 thread and one OpenMP thread per CPU of this process's
    affinity mask, scaled to filter steps/s of the n particles the bench line
    ran (per GPU at N>1).  `value` is the all-core rate of the config's own
    filter; the rate at OMP_NUM_THREADS threads (the box's CPU share) is
    reported beside it, and a PHD-only leg of the same shape (config 3's CPHD
    oracle evaluates the Ψ1d inner products directly).  births: the GPU line's
    step placed the scan's births (CPHD), so the oracle legs do too."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    cores = max(1, len(aff))
    omp_env = os.environ.get("OMP_NUM_THREADS")
    omp = max(1, min(cores, int(omp_env))) if omp_env and omp_env.isdigit() else 0
    cfg = __import__("phdslam").preset(config_id)[0]
    cphd = cfg.filterType == 1
    legs = [False, True] if cphd else [False]
    per = budget_s / ((3 if omp and omp not in (1, cores) else 2) * len(legs))
    res = {}
    for phd_only in legs:
        r1, reps1, ns1, _, G, M, dt1, _ = _oracle_rate(config_id, n, 1, per, phd_only, births)
        rc, repsc, nsc, _, _, _, dtc, used = _oracle_rate(config_id, n, cores, per, phd_only, births) if cores > 1 else \
            (r1, reps1, ns1, n, G, M, dt1, 1)
        res[phd_only] = (r1, reps1, ns1, dt1, rc, repsc, nsc, dtc, used)
    r1, reps1, ns1, dt1, rc, repsc, nsc, dtc, used = res[False]
    out = {"value": rc / n, "unit": "steps/s", "cores": used, "kind": "port", "value_1thread": r1 / n,
           "cpu_model": _cpu_model(), "affinity": _ranges(aff), "affinity_cpus": len(aff),
           "omp_num_threads_env": omp_env,
           "build": "oracle/liboracle_fast.so: g++ -O3 -march=x86-64-v3 -fopenmp -ffp-contract=off",
           "sample": f"oracle predict{'+births' if births else ''}+update+normalize ({'CV + CPHD' if cphd else 'PHD'}) on {ns1}-/{nsc}-particle "
                     f"samples of the config (G={G}, M={M}): 1 thread {reps1} reps in {dt1:.1f}s; {used} OpenMP "
                     f"threads {repsc} reps in {dtc:.1f}s; particle-updates/s scaled to N={n} (the particles per GPU "
                     f"this line ran)"}
    if omp and omp not in (1, cores):
        ro, repso, nso, _, _, _, dto, usedo = _oracle_rate(config_id, n, omp, per, False, births)
        out["omp_env_leg"] = {"value": ro / n, "threads": usedo,
                              "sample": f"{usedo} OpenMP threads (OMP_NUM_THREADS) {repso} reps x {nso} particles "
                                        f"in {dto:.1f}s"}
    if cphd:
        out["sample"] += ("; the CPHD oracle evaluates each measurement's <Psi1d,p> by the direct O(Nmax M^2) "
                          "log-sum-exp (scphd_cpu.cpp cphd_terms), the GPU by the closed form (DESIGN D9)")
        p1, preps1, pns1, pdt1, pc, prepsc, pnsc, pdtc, _ = res[True]
        out["phd_only"] = {"value": pc / n, "value_1thread": p1 / n,
                           "sample": f"same shape with filter_type 0: 1 thread {preps1} reps x {pns1} particles in "
                                     f"{pdt1:.1f}s; {used} threads {prepsc} reps x {pnsc} in {pdtc:.1f}s"}
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


TIMING_STRIDE = 8  # the update-timing events sample at most every 8th timed update


def copy_bandwidth(dev, mib=1024, reps=10):
    """Achievable HBM ceiling: device-to-device copy of a 1 GiB buffer
    (read + write bytes / time), HIP events on the current stream."""
    import torch
    a = torch.empty(mib << 20, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    gbs = 2 * a.numel() * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    return gbs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=3,
                    help="BASELINE.json config (1..5, SURVEY.md §8(d)); 1 = the CPU oracle over the reference's data")
    ap.add_argument("--particles", type=int, default=0, help="override particles per GPU")
    ap.add_argument("--threads", type=int, default=0, help="threads per particle of the fused update (0 = auto)")
    ap.add_argument("--form", type=int, default=0, help="PHD update form: 0 auto, 1 one fused launch, 2 split (A + C)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (gloo only to rehearse N>1 on one GPU)")
    ap.add_argument("--mode", choices=["replay", "sequence"], default="replay",
                    help="replay: one fixed measurement set (the reference's profile replay, main.cpp:1314-1321); "
                         "sequence: a fresh measurement set every step, uploaded inside the timed loop as run_synth "
                         "does (main.cpp:1233,1271)")
    ap.add_argument("--block-records", type=int, default=4,
                    help="sharded step: particle records per peer in the fixed all-to-all blocks")
    ap.add_argument("--births", type=int, default=-1, choices=[-1, 0, 1],
                    help="the step's births of the previous scan (phd_set_step_births): -1 with the filter type "
                         "(CPHD: on, the reference's loop), 0 off (diagnostic A/B only), 1 on")
    ap.add_argument("--no-config4-model", action="store_true",
                    help="skip the companion line of config 4's own model (Ackerman + PHD, 4096 particles per GPU "
                         "of one filter) that config-3 runs report beside their value")
    ap.add_argument("--transport", choices=["cxx", "torch"], default="cxx",
                    help="sharded step: cxx = one C call per step (phdslam.dist.GroupRank: the C++ host over its own "
                         "RCCL communicator, include/phd_group.h); torch = phdslam.dist.ShardedFilter (the phases "
                         "issued from Python, collectives through torch.distributed)")
    ap.add_argument("--force-sharded", action="store_true",
                    help="run the sharded step (phdslam.dist.ShardedFilter: all-gather + all-to-all over "
                         "torch.distributed, RCCL for backend nccl) even at one rank")
    args = ap.parse_args()
    if args.config == 1:  # BASELINE configs[0]: the reference's CPU-only case (no GPU leg)
        config1_line(args)
        return

    import numpy as np
    import torch
    import phdslam

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or args.force_sharded:
        import torch.distributed as dist
        ndev = torch.cuda.device_count()
        local_dev = local_rank % ndev  # ndev < world only in a gloo rehearsal on one GPU
        torch.cuda.set_device(local_dev)
        if "MASTER_ADDR" not in os.environ:  # one rank without a launcher
            import socket
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]), RANK="0",
                              WORLD_SIZE="1", LOCAL_RANK="0")
            sk.close()
        # RCCL may print a version banner on stdout when the communicator comes up:
        # keep stdout for the one JSON line (the banner goes to stderr)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(args.backend, device_id=torch.device("cuda", local_dev)
                                    if args.backend == "nccl" else None)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    else:
        local_dev = 0
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local_dev)

    cfg, n, G, M, df = phdslam.preset(args.config)
    if args.config == 4 and world > 1:
        n = n // world  # config 4 is quoted as a whole 8-GPU job (4096 per GPU)
    if args.particles:
        n = args.particles
    from phdslam.scenario import SEED_BASE
    seed = SEED_BASE + args.config
    # every rank holds a shard of one filter: the same prior scenario (drawn from
    # one posterior), distinct predict noise via the global particle index
    _, poses, lw, maps, offs, z = phdslam.config_scenario(args.config, n=n, G=G, M=M, seed=seed)
    # capacities sized to the replay workload (phdslam.scenario.bench_capacities,
    # the set tests/test_gpu_parity.py::test_cphd_update_bench_configuration holds
    # to the oracle); an overflow in the untimed warm-up switches to the roomier
    # set before anything is timed, and the timed region is checked again after
    from phdslam.scenario import bench_capacities

    def make_filter(wide):
        f = phdslam.PHDFilter(n, cfg, device=dev.index, **bench_capacities(args.config, G, M, wide))
        f.set_seed(seed)
        f.set_step_births(args.births)
        f.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        f.load(poses, lw, maps, offs)
        f.set_measurements(z)
        f.set_replay(True)
        if args.form:
            f.set_update_form(args.form)
        if args.threads:
            f.set_update_threads(args.threads)
        f.set_check_each_update(False)
        return f

    wide = False
    f = make_filter(wide)
    sharded = make_sharded(args, f, dist, dev) if dist is not None else None

    control = (2.0, 0.05)
    motion_ack = cfg.motionType == 1
    # sequence mode: S synthetic measurement sets (the replay set with fresh
    # range / bearing noise and fresh clutter), one set_measurements per step
    zseq = None
    if args.mode == "sequence":
        rng = np.random.default_rng(seed + 1)
        zseq = []
        for _ in range(16):
            zk = z.copy()
            zk["range"] = np.abs(zk["range"] + rng.normal(0, cfg.stdRange, len(zk))).astype(np.float32)
            zk["bearing"] = (zk["bearing"] + rng.normal(0, cfg.stdBearing, len(zk))).astype(np.float32)
            clut = rng.random(len(zk)) < 0.25
            zk["range"][clut] = rng.uniform(0, cfg.maxRange, int(clut.sum()))
            zk["bearing"][clut] = rng.uniform(-np.pi, np.pi, int(clut.sum()))
            zseq.append(zk)

    def one_step(k):
        if zseq is not None:
            f.set_measurements(zseq[k % len(zseq)])
        if sharded is not None:
            sharded.step(control if motion_ack else None, k)
        else:
            _step_async(f, control, motion_ack, k)

    # the achievable-bandwidth reference of the roofline (a 1 GiB device copy)
    copy_gbs = copy_bandwidth(dev)
    # GPU clock warm-up before the warm-up steps: a cold GPU ramps its shader
    # clock over tens of ms, so after only the driver's 5 warm-up steps (1.5 ms
    # of work) its first 20 timed steps run ~6 % below the steady state (20
    # steps after 5 warm-up steps: 3 274 / 3 264 steps/s; after 100: 3 449 /
    # 3 472; after 5 with this burst: 3 417 / 3 435 — profiles/r06_warm_probe.txt).
    # Unrelated matrix work (not filter steps: the warm-up stays W steps and the
    # timed region exactly K); PHD_BENCH_CLOCK_WARMUP=0 skips it
    spin = int(os.environ.get("PHD_BENCH_CLOCK_WARMUP", "40"))
    t_spin = time.perf_counter()
    if spin > 0:
        x = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
        for _ in range(spin):
            x = (x @ x).clamp_(-1, 1)
        torch.cuda.synchronize(dev)
        del x
    t_spin = time.perf_counter() - t_spin
    for k in range(args.warmup):
        one_step(k)
    torch.cuda.synchronize(dev)
    try:
        f.check_errors()
    except phdslam.PHDError:
        if sharded is not None:
            raise
        f.close()
        wide = True
        f = make_filter(wide)
        for k in range(args.warmup):
            one_step(k)
        torch.cuda.synchronize(dev)
        f.check_errors()
    # HIP events around a sample of the timed region's updates: every
    # max(TIMING_STRIDE, steps / 16)-th (each event record costs the stream
    # ~2.4 us: timing all of them slowed the timed steps by ~2 %, and a stride
    # of 1 at the driver's 20 steps had cost its line 7 %); 20 steps sample 3
    # updates, 200 steps 17
    stride = max(TIMING_STRIDE, args.steps // 16)
    f.enable_timing(args.steps, stride=stride)
    rs0 = f.resample_count()
    # slow-path counters of the timed steps only (data-dependent fallbacks must
    # not hide behind the replay number): serial-greedy merges, pair-list
    # overflow walks, particle-updates with an error status bit
    f.merge_fallbacks()
    f.merge_pair_overflows()
    f.status_errors()
    st0 = None
    if sharded is not None:
        sharded.flush()
        st0 = dict(sharded.stats)  # count the timed steps only
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(args.warmup + k)
    if sharded is not None:
        sharded.flush()  # the last step's plan (records beyond the blocks, if any)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    upd_ms, upd_cnt = f.update_timing()
    resamples = f.resample_count() - rs0
    slow = {"merge_fallbacks": f.merge_fallbacks(), "merge_pair_overflows": f.merge_pair_overflows(),
            "status_errors": f.status_errors(), "particle_updates": n * args.steps}
    f.check_errors()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # algorithmic bytes of one fused update launch: prior sizes in (with the
    # step's births), written out-slab sizes
    births = f.step_births()
    sizes_out = f.slab_sizes()
    sizes_in = np.diff(offs) + (int(np.sum(z["label"] == 0)) if births and cfg.labeledMeasurements else len(z) if births
                                else 0)
    B = algorithmic_bytes(sizes_in, sizes_out, M)
    avg_upd_s = (upd_ms / max(upd_cnt, 1)) / 1e3
    achieved = B / avg_upd_s / 1e9 if avg_upd_s > 0 else 0.0  # (0: a diagnostic build without timing events)

    total_particles = n * world
    # Weak scaling (every config but 4): each GPU steps its own config-sized
    # particle batch, so the whole job completes `world` config-steps per step.
    # Config 4 is one fixed 32768-particle filter split over the GPUs (strong).
    strong = args.config == 4 and world > 1
    value = (1 if strong else world) * args.steps / elapsed
    line = {
        "metric": "PHD update steps/sec at N_particles x N_gm x N_meas; achieved HBM GB/s vs roofline",
        "value": round(value, 2),
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (deterministic replay scenario, SURVEY.md §8(d))" if args.mode == "replay" else
                "synthetic (replay prior, a fresh measurement set uploaded every step, SURVEY.md §8(d) sequence mode)",
        "config": {"workload": f"config{args.config}: {total_particles} particles x {G} GM x {M} meas, "
                               f"{'Ackerman' if motion_ack else 'CV'} predict"
                               f"{' + births of the previous scan (' + str(M) + ' per particle after its ' + str(G) + ' prior components; replay: of the replayed scan)' if births else ''}"
                               f" + static {'CPHD' if cfg.filterType == 1 else 'PHD'} update, {args.mode}",
                   "step_births": births,
                   "particles": total_particles, "particles_per_gpu": n, "gm_components": G,
                   "measurements": M,
                   "parallelism": (f"particle-shard x{world} ({args.backend})" if sharded is not None else "single GPU"),
                   "mode": args.mode,
                   "particle_steps_per_s": round(args.steps / elapsed * total_particles, 1),
                   "filter_steps_per_s": round(args.steps / elapsed, 2)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": _update_kernels(f, cfg), "avg_kernel_ms": round(avg_upd_s * 1e3, 5), "timed_updates": upd_cnt,
                     "algorithmic_bytes_per_launch": B},
    }
    # HBM traffic per update and the dominant kernel's VALU / LDS issue
    # utilisation from the committed PMC passes of this config
    # (scripts/gpu_round_pmc.sh -> scripts/pmc_report.py; gfx950 FETCH correction)
    # (measured in replay mode: not attached to a sequence-mode line)
    # (a file per particle count, traffic_c<C>_n<n>.json, else the config's
    # default-shape file, only when this run has the config's default shape)
    def _pmc_file(kind):
        p = os.path.join(REPO, "profiles", f"{kind}_c{args.config}_n{n}.json")
        if os.path.exists(p):
            return p
        p = os.path.join(REPO, "profiles", f"{kind}_c{args.config}.json")
        return p if n == phdslam.preset(args.config)[1] else ""

    tpath = _pmc_file("traffic")
    if tpath and os.path.exists(tpath) and args.mode == "replay":
        with open(tpath) as fh:
            t = json.load(fh)
        line["roofline"]["traffic"] = round(float(t["bytes_per_launch"]))
        line["roofline"]["traffic_source"] = os.path.relpath(tpath, REPO)
    ppath = _pmc_file("pmc")
    if ppath and os.path.exists(ppath) and args.mode == "replay":
        with open(ppath) as fh:
            pm = json.load(fh)
        line["roofline"]["valu_util"] = pm.get("valu_util")
        line["roofline"]["lds_util"] = pm.get("lds_util")
        line["roofline"]["update_valu_util"] = pm.get("update_valu_util")
        line["roofline"]["dominant_kernel"] = pm.get("dominant_kernel")
        line["roofline"]["util_source"] = os.path.relpath(ppath, REPO)
    (line["config"]["update_threads"], line["config"]["update_lds_bytes"],
     line["config"]["update_resident_workgroups"]) = f.update_threads()
    line["config"]["update_split"] = f.update_form()
    line["config"]["resample_rate"] = round(resamples / args.steps, 4)
    line["config"]["slow_paths"] = slow
    caps = f.capacity
    line["config"]["capacities"] = {"map": caps.map_capacity, "candidates": caps.candidate_capacity,
                                    "survivors": caps.survivor_capacity, "measurements": caps.max_measurements,
                                    "overflow_fallback": wide}
    line["roofline"]["copy_ceiling_gbs"] = round(copy_gbs, 1)
    line["config"]["gpu_clock_warmup"] = (f"{spin} bf16 8192^3 matrix products ({1e3 * t_spin:.0f} ms) before the "
                                          f"{args.warmup} warm-up steps" if spin > 0 else "none")
    if sharded is not None:
        st = {k: v - st0[k] for k, v in sharded.stats.items()}
        line["config"]["transport"] = args.transport if args.backend == "nccl" else "torch"
        line["config"]["resamples"] = st["resamples"]
        line["config"]["migrated_particles"] = st["migrated"]
        line["config"]["migrated_records"] = st["records"]
        line["config"]["block_records"] = sharded.K
        line["config"]["overflow_records"] = st["overflow_records"]
        line["config"]["pending_slots"] = st["pending_slots"]
        if hasattr(sharded, "close"):
            sharded.close()
    if args.config == 3 and not args.no_config4_model:
        # the north-star ratio is config 4's own model on 8 GPUs
        # (Ackerman + PHD, one 32 768-particle filter) over config 3 on one GPU;
        # the driver's scaling curve is computed from `value` (config-3 shards),
        # so config 4's model is measured beside it at every N
        f.close()
        f = None
        try:
            line["config4_model"] = _config4_model(args, dist, dev, world)
        except Exception as e:  # report, never fake (the main line stands)
            line["config4_model"] = {"value": None, "error": str(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # (N = 1 only: the bounded host sample)
        try:
            line["cpu_baseline"] = cpu_baseline(args.config, n, args.cpu_budget, births=bool(births))
        except Exception as e:  # report, never fake
            line["cpu_baseline"] = {"value": None, "error": str(e)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if f is not None:
        f.close()
    if dist is not None:
        dist.destroy_process_group()


def config1_line(args):
    """Config 1 as BASELINE.json configs[0] states it: the CPU oracle alone
    (oracle/liboracle_fast.so) in the reference's loop (main.cpp:1178-1312:
    predict, update when |Z| > 0, nEff, resample when nEff <= 0.5) over the
    reference's own data (python/controls_synth.txt + measurements_synth.txt,
    tests/golden/config1_data.npz: 1 135 scans, 1 134 controls) at 64
    particles with the G-cap-64 policy (oracle/config1_loop.py), every scan,
    once on 1 thread and once on every CPU of the affinity mask.  No GPU runs
    and no warm-up: `steps` is the number of scans, timed whole."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import phdslam
    import config1_loop as L
    cfg, n, G, M, _ = phdslam.preset(1)
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    # all cores = one OpenMP thread per CPU of the affinity mask, at most one per
    # particle (the oracle's parallel loops are over the 64 particles: 256
    # threads on the GPU box's 256 CPUs ran 7.8 steps/s against 59.9 on one —
    # fork / join of 256 threads per call); OMP_NUM_THREADS' count (the box's
    # CPU share) beside it
    n_all = max(1, min(len(aff), n))
    omp_env = os.environ.get("OMP_NUM_THREADS")
    omp = max(1, min(int(omp_env), n_all)) if omp_env and omp_env.isdigit() else 0
    legs = {}
    for threads in sorted({1, n_all} | ({omp} if omp else set())):
        state, dt, S, rs = L.run(cfg, n=n, seed=SEED_C1, threads=threads)
        legs[threads] = (S / dt, dt, S, rs, int(np.diff(state[3]).max(initial=0)))
    # value: the fastest leg (on the GPU box the 16-CPU share of OMP_NUM_THREADS
    # beats one thread per particle: 64 threads oversubscribe it)
    best = max(legs, key=lambda t: legs[t][0])
    allc = legs[best]
    one = legs[1]
    line = {
        "metric": "PHD update steps/sec at N_particles x N_gm x N_meas; achieved HBM GB/s vs roofline",
        "value": round(allc[0], 2), "unit": "steps/s", "n_gpus": 0, "steps": allc[2], "warmup": 0,
        "ms_per_step": round(1e3 * allc[1] / allc[2], 3), "higher_is_better": True, "scaling": "none",
        "vs_baseline": None, "dtype": "f32",
        "data": "the reference's own data files (python/controls_synth.txt, python/measurements_synth.txt)",
        "config": {"workload": f"config1: {n} particles x G cap {L.G_CAP} x {M} meas (mean per scan), Ackerman "
                               f"predict + static PHD update, the reference's loop, CPU oracle only "
                               f"(BASELINE configs[0]; no GPU leg)",
                   "particles": n, "g_cap": L.G_CAP, "scans": allc[2], "resamples": allc[3],
                   "max_map_size": allc[4], "parallelism": "OpenMP over particles"},
        "roofline": None,
        "cpu_baseline": {"value": round(allc[0], 2), "unit": "steps/s", "cores": best, "kind": "port",
                         "value_1thread": round(one[0], 2), "seconds_1thread": round(one[1], 2),
                         "seconds_all_cores": round(legs[n_all][1], 2), "value_all_cores": round(legs[n_all][0], 2),
                         "nproc": os.cpu_count(),
                         "affinity": _ranges(aff), "affinity_cpus": len(aff), "cpu_model": _cpu_model(),
                         "omp_num_threads_env": omp_env,
                         "legs": {str(k): round(v[0], 2) for k, v in sorted(legs.items())},
                         "build": "oracle/liboracle_fast.so: g++ -O3 -march=x86-64-v3 -fopenmp -ffp-contract=off",
                         "sample": f"every scan of the data ({allc[2]} scans), predict + update + normalize + nEff + "
                                   f"resample ({allc[3]} resamples) + G cap; 1 thread, {n_all} OpenMP threads (one per "
                                   f"CPU of the affinity mask, at most one per particle)"
                                   + (f" and OMP_NUM_THREADS={omp}" if omp and omp not in (1, n_all) else "")
                                   + f"; value: the fastest leg ({best} threads)"},
    }
    print(json.dumps(line), flush=True)


SEED_C1 = 5  # the predict / resample Philox seed of config 1's loop (tests/test_gpu_parity.py uses the same)


def _config4_model(args, dist, dev, world):
    """Config 4's own model beside a config-3 line: Ackerman predict + static
    PHD update (its M births in the update array), 4 096 particles per GPU of
    ONE filter (at N = 8 the 32 768 x 512 x 64 job of configs[3]), the same
    step (sharded at N > 1: all-gather + all-to-all), warm-up and timed steps
    as the main line; the max over ranks of the timed region."""
    import numpy as np  # noqa: F401
    import torch
    import phdslam
    from phdslam.scenario import SEED_BASE, bench_capacities
    cid = 4
    cfg, n_job, G, M, _ = phdslam.preset(cid)
    n = n_job // 8  # per GPU
    seed = SEED_BASE + cid
    _, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=n, G=G, M=M, seed=seed)
    f = phdslam.PHDFilter(n, cfg, device=dev.index, **bench_capacities(cid, G, M, False))
    f.set_seed(seed)
    f.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    f.load(poses, lw, maps, offs)
    f.set_measurements(z)
    f.set_replay(True)
    f.set_check_each_update(False)
    sharded = make_sharded(args, f, dist, dev) if dist is not None else None
    control = (2.0, 0.05)

    def one_step(k):
        if sharded is not None:
            sharded.step(control, k)
        else:
            _step_async(f, control, True, k)

    for k in range(args.warmup):
        one_step(k)
    torch.cuda.synchronize(dev)
    f.check_errors()
    f.merge_fallbacks()
    f.merge_pair_overflows()
    f.status_errors()
    st0 = None
    if sharded is not None:
        sharded.flush()
        st0 = dict(sharded.stats)  # count the timed steps only
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(args.warmup + k)
    if sharded is not None:
        sharded.flush()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    slow = {"merge_fallbacks": f.merge_fallbacks(), "merge_pair_overflows": f.merge_pair_overflows(),
            "status_errors": f.status_errors()}
    f.check_errors()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    nt, lds, res = f.update_threads()
    out = {"workload": f"config4: {n * world} particles x {G} GM x {M} meas (one filter, {n} per GPU), "
                       f"Ackerman predict + static PHD update, replay",
           "filter_steps_per_s": round(args.steps / elapsed, 2),
           "particle_steps_per_s": round(args.steps / elapsed * n * world, 1),
           "ms_per_step": round(1e3 * elapsed / args.steps, 4), "steps": args.steps, "n_gpus": world,
           "update_threads": nt, "update_split": f.update_form(), "update_resident_workgroups": res,
           "slow_paths": slow}
    if sharded is not None:  # (records beyond the fixed blocks go point to point, their slots re-updated)
        st = {k: v - st0[k] for k, v in sharded.stats.items()}
        out.update(resamples=st["resamples"], migrated_particles=st["migrated"], migrated_records=st["records"],
                   overflow_records=st["overflow_records"], block_records=sharded.K,
                   transport=args.transport if args.backend == "nccl" else "torch")
        if hasattr(sharded, "close"):
            sharded.close()
    f.close()
    return out


def make_sharded(args, f, dist, dev):
    """The sharded step over the torch.distributed group: the C++ host's rank
    (one C call per step, its own RCCL communicator) or the Python
    ShardedFilter (--transport torch; gloo rehearsals).  Both run the same plan
    bit for bit (tests/test_gpu_parity.py::test_group_rank_matches_sharded_filter)."""
    if args.transport == "cxx" and args.backend == "nccl":
        from phdslam.dist import GroupRank
        # (its communicator comes up here: any RCCL banner goes to stderr, as
        # for the torch.distributed group's)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            return GroupRank(f, dist, dev, block_records=args.block_records)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    from phdslam.dist import ShardedFilter
    return ShardedFilter(f, dist, dev, block_records=args.block_records)


def _update_kernels(f, cfg):
    """The launches timed as one update (HIP events around them)."""
    nt = f.update_threads()[0]
    if cfg.filterType == 1:
        return f"k_update_cphd_a_{nt}+k_cphd_terms+k_update_cphd_c_{nt}"
    if f.update_form():
        return f"k_update_phd_a_{nt}+k_update_phd_c_{nt}"
    return f"k_update_fused_{nt}"


def _step_async(f, control, motion_ack, k):
    """phd_step without host read-backs (device-side resample decision)."""
    import ctypes
    from phdslam import _lib
    from phdslam.types import AckermanControl
    u = ctypes.byref(AckermanControl(float(control[1]), float(control[0]))) if motion_ack else None
    _lib.check(_lib.lib().phd_step(f.handle, u, 1, int(k), None, None), "phd_step")


if __name__ == "__main__":
    main()
