#!/usr/bin/env python3
"""Benchmark: frame-pairs/sec of the DIS hot path at 1920x1080 preset=medium.

One step = one call of the whole path (pyramid -> coarse-to-fine patch search
-> densify -> upsample/crop) over a batch of synthetic u8 frame pairs already
resident in HBM; outputs stay in HBM. Pairs shard across ranks (one process
per GPU, launched by torch.distributed.run); there is no collective on the data
path -- only the barrier and the max-over-ranks timing reduction.

Prints ONE JSON line on rank 0 (contract in the task statement); extra fields:
`roofline` for the dominant kernel (the finest-level patch-search launch,
k_search8, ~60% of the step), which is bound by VALU issue -- its f32
arithmetic must stay separately rounded (no FMA) to match the reference bit for
bit -- with its HBM figures alongside; `cpu_baseline` (the C oracle in one
process per host core, <= 16, plus a one-core sample) and `max_epe_vs_oracle`.
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import disflow  # noqa: E402

METRIC = "frame-pairs/sec at 1920x1080 preset=medium, 1/2/4/8 GPUs; max EPE vs reference"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# f32 VALU peak for non-fused operations: the 157.3 TFLOP/s vector-f32 peak
# (MI355X_MICROARCH.md) counts an FMA as 2 FLOPs; the reference's separately
# rounded mul/add forbid FMA, so one lane-operation per FLOP: 157.3 / 2.
VALU_PEAK_TFLOPS = 78.6
FMA_PEAK_TFLOPS = 157.3  # vector f32 with FMA = 2 ops (MI355X_MICROARCH.md)
WARMUP_FLOOR_S = 0.5  # untimed GPU work before the timed region, whatever --warmup is


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32, help="pairs per GPU per step")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--preset", default="medium", choices=[p.name.lower() for p in disflow.Preset])
    ap.add_argument("--streams", type=int, default=0, help="sub-batch streams per step (0 = library default)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline sample budget")
    ap.add_argument("--cpu-workers", type=int, default=0, help="CPU-baseline host processes (0 = all, <= 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="process group backend for N > 1 (nccl = RCCL; "
                    "gloo only to rehearse several ranks on one GPU)")
    ap.add_argument("--no-kernel-timing", action="store_true", help="diagnostic: no per-launch events")
    ap.add_argument("--default-stream", action="store_true", help="diagnostic: issue the calls on the default stream")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the extra two-batches-in-flight measurement (reported beside, never as, value)")
    ap.add_argument("--no-tolerance-mode", action="store_true",
                    help="skip the extra DIS_PRECISION_FMA measurement (reported beside, never as, value)")
    ap.add_argument("--warmup-floor", type=float, default=WARMUP_FLOOR_S,
                    help="seconds of untimed steps at least (after the W warmup steps); 0 under a profiler")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: shard plan, gather + checksum verification over gloo with stand-in flows, "
                         "and the line's schema (value null); use with --dist-backend gloo for N > 1")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per search launch (from tools/pmc_traffic.py)")
    return ap.parse_args()


def make_pairs(seeds, W, H):
    def one(s):
        return disflow.synth_pair(int(s), W, H)

    with cf.ThreadPoolExecutor(max_workers=min(16, len(seeds))) as ex:
        res = list(ex.map(one, seeds))
    return np.stack([a for a, _ in res]), np.stack([b for _, b in res])


CPU_WORKER_CAP = 16  # the GPU box's CPU share per GPU (gpurun: 16); nproc shows the whole host


def oracle_lib_for_baseline():
    """The -O3 build of the oracle (the CPU baseline is the C
    restatement at -O3, single-threaded per pair); -O2 checker build otherwise."""
    o3 = os.path.join(ROOT, "oracle", "libdis_oracle_o3.so")
    return o3 if os.path.exists(o3) else os.path.join(ROOT, "oracle", "libdis_oracle.so")


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def physical_cores():
    """Distinct (physical id, core id) pairs in /proc/cpuinfo (SMT siblings
    counted once); None if the file does not say."""
    try:
        cores, phys = set(), None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                cores.add((phys, line.split(":", 1)[1].strip()))
        return len(cores) or None
    except OSError:
        return None


_CPU_POOL = None  # (I0, I1) stacks of the CPU baseline's input pairs, shared with the forked workers


def _cpu_worker(args):
    """One host process of the CPU baseline: oracle pairs (from the pre-generated
    pool, like the GPU's HBM-resident inputs) until the deadline."""
    k0, step, pfields, deadline = args
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["DIS_ORACLE_LIB"] = oracle_lib_for_baseline()
    import oracle_binding

    params = disflow.Params(**pfields)
    I0s, I1s = _CPU_POOL
    # worker w takes pairs w, w + step, w + 2 step, ... of the global sequence
    # and cycles the pool by its own count (k0 + n*step modulo a
    # pool of `step` pairs would revisit one pair forever)
    n = 0
    while True:
        k = (k0 + n) % len(I0s)
        oracle_binding.calc_from_params(I0s[k], I1s[k], params)
        n += 1
        if time.time() >= deadline:
            return n


def cpu_baseline(params, W, H, budget_s, workers):
    """The C oracle on a bounded sample of the workload: one
    core (latency), then `workers` host processes, one pair at a time each,
    like the reference's single-threaded per-pair path (throughput). The input
    pairs are generated before the clock starts (r05: generating them inside
    the timed loop had cost as much as the oracle itself at 1080p). Runs
    before the GPU is initialised, so the worker processes are plain forks."""
    import multiprocessing as mp

    global _CPU_POOL
    _CPU_POOL = make_pairs(range(max(1, min(workers, 16))), W, H)
    pf = dict(vars(params))
    t0 = time.time()
    n1 = _cpu_worker((0, 1, pf, t0 + budget_s / 3))
    t1 = time.time() - t0
    out = {"single_core": {"value": n1 / t1, "pairs": n1}}
    if workers > 1:
        ctx = mp.get_context("fork")
        t0 = time.time()
        deadline = t0 + 2 * budget_s / 3
        # close + join (not the context manager, whose exit terminate()s the
        # workers: under rocprofv3 that SIGTERM printed an abort trace)
        pool = ctx.Pool(workers)
        try:
            ns = pool.map(_cpu_worker, [(w, workers, pf, deadline) for w in range(workers)])
        finally:
            pool.close()
            pool.join()
        out.update(value=sum(ns) / (time.time() - t0), cores=workers, pairs=sum(ns))
    else:
        out.update(value=n1 / t1, cores=1, pairs=n1)
    return out


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(a):
    """`--gpus N > 1` without a launcher: start the N ranks ourselves as
    `torch.distributed.run` children (one process per GPU, rendezvous on
    127.0.0.1) and exit with their status. Runs before anything touches the
    GPU (this process only counts devices), so nothing is re-exec'd."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench: --gpus {a.gpus} without WORLD_SIZE: launching {a.gpus} ranks under torch.distributed.run",
          file=sys.stderr, flush=True)
    sys.exit(subprocess.run(cmd).returncode)


def check_world(a, world, rank):
    """The line must describe the ranks that really ran: --gpus == WORLD_SIZE,
    and under nccl (RCCL) one distinct GPU per local rank."""
    if a.gpus != world:
        raise SystemExit(f"bench: --gpus {a.gpus} but WORLD_SIZE {world}: refusing to report a "
                         f"{world}-rank measurement as {a.gpus} GPUs")
    if a.dry_run and world > 1 and a.dist_backend != "gloo":
        raise SystemExit("bench: --dry-run runs on the CPU: use --dist-backend gloo")
    if a.dist_backend == "nccl" and world > 1 and not a.dry_run:
        ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        if lws > ndev:
            raise SystemExit(f"bench: {lws} local ranks but {ndev} visible GPU(s) under nccl: ranks would "
                             f"share a GPU (use --dist-backend gloo only to rehearse that)")


def gather_and_verify(out, B, rank, world, backend, sync=lambda: None, on_full=None):
    """The path's one collective (SURVEY.md 8e, config 4 "RCCL gather only"):
    every rank's (B, H, W, 2) flows gathered to rank 0 in pair order
    (disflow.multi.gather_flow_tensor; RCCL for nccl, host tensors under gloo),
    then verified: each rank's bit-level checksum of its own shard against rank
    0's checksum of that shard of the gathered tensor. A failure on any rank is
    shared (one all-reduce) before the checksum collective, so every rank skips
    it together. Returns the line's `gather` object on rank 0."""
    import disflow.multi as multi
    tg = time.perf_counter()
    full = None
    try:
        full = multi.gather_flow_tensor(out, world * B, rank, world)
        sync()
        gather_err = None
    except (RuntimeError, MemoryError) as e:  # reported in the line; the timed result stands
        full, gather_err = None, f"{type(e).__name__}: {e}"
    tg = time.perf_counter() - tg
    any_err = multi.any_rank_failed(gather_err is not None, world)
    if any_err and gather_err is None:
        gather_err = "another rank's gather failed"
    sums = multi.gather_checksums(multi.flow_checksum(out), rank, world) if not any_err else None
    if rank != 0:
        return None
    if any_err:
        return {"error": gather_err, "world_size": world}
    if int(full.shape[0]) != world * B:
        raise SystemExit(f"bench: gathered {full.shape[0]} pairs, expected {world * B}")
    got = [multi.flow_checksum(full[r * B:(r + 1) * B]) for r in range(world)]
    verified = all(torch.equal(g.cpu(), e.cpu()) for g, e in zip(got, sums))
    if not verified:
        raise SystemExit("bench: gathered flows differ from the ranks' own flows")
    if on_full is not None:
        on_full(full)
    nbytes = (world - 1) * out.numel() * out.element_size()  # bytes that crossed xGMI
    return {"ms": tg * 1e3, "bytes_received": nbytes, "GB_per_s": nbytes / tg / 1e9,
            "pairs": int(full.shape[0]), "verified": verified, "world_size": world,
            "backend": "nccl (RCCL)" if backend == "nccl" else backend}


DRY_HW = (6, 8)  # --dry-run flow fields: tiny, so an 8-rank gloo rehearsal stays cheap


def dry_run(a, rank, world):
    """--dry-run (CPU, no GPU call): the multi-rank plumbing of the bench line
    exactly as a real N-rank run takes it -- the rank layout, the per-rank
    shard of the global batch, the gather + checksum verification of
    gather_and_verify over the process group (gloo here) -- with a
    deterministic stand-in for the flows (tiny fields, a function of the
    global pair index, so rank 0 also checks the pair order) -- and the line's
    schema with `value` null. DIS_BENCH_DRY_FAIL=check|alloc makes rank 0's
    receive-buffer check or allocation fail (tests)."""
    import disflow.multi as multi
    B = a.batch
    if world > 1:
        torch.distributed.init_process_group("gloo")
    fail = os.environ.get("DIS_BENCH_DRY_FAIL")
    if fail == "check":
        multi.check_gather_fits = lambda nbytes, free, margin=0.9: (_ for _ in ()).throw(
            MemoryError("dry-run: injected rank-0 receive-buffer check failure"))
    elif fail == "alloc" and rank == 0:
        real_empty = torch.empty
        torch.empty = lambda *s, **k: (_ for _ in ()).throw(RuntimeError("dry-run: injected allocation failure")) \
            if len(s) and isinstance(s[0], tuple) and s[0][0] == world else real_empty(*s, **k)
    h, w = DRY_HW
    a0, a1 = multi.shard_bounds(world * B, rank, world)
    ids = torch.arange(a0, a1, dtype=torch.float32).view(-1, 1, 1, 1)
    grid = torch.arange(h * w * 2, dtype=torch.float32).view(1, h, w, 2)
    out = ids * 1000.0 + grid  # pair k: k*1000 + position
    order = {}

    def check_order(full):  # rank 0: pair k of the gathered tensor is global pair k
        want = torch.arange(world * B, dtype=torch.float32).view(-1, 1, 1, 1) * 1000.0 + grid
        order["pair_order_ok"] = bool(torch.equal(full, want))

    gather = gather_and_verify(out, B, rank, world, "gloo", on_full=check_order) if world > 1 else None
    if fail == "alloc" and rank == 0:
        torch.empty = real_empty
    if rank == 0:
        if gather is not None and "error" not in gather:
            gather.update(order)
        plan = [list(multi.shard_bounds(world * B, r, world)) for r in range(world)]
        line = {"metric": METRIC, "value": None, "unit": "frame-pairs/s", "n_gpus": world, "steps": a.steps,
                "warmup": a.warmup, "dry_run": True,
                "config": {"workload": f"{a.width}x{a.height} preset={a.preset}, {B} pairs/GPU/step, "
                                       "inputs+outputs in HBM",
                           "width": a.width, "height": a.height, "preset": a.preset, "global_batch": world * B,
                           "parallelism": f"pairs sharded over {world} rank(s), no data-path collective"},
                "shards": plan, "gather": gather,
                "note": f"--dry-run: no GPU work; stand-in flows of {h}x{w} per pair through the real gather and "
                        "checksum verification (gloo); value is not measured"}
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(a)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_world(a, world, rank)
    if os.environ.get("DIS_BENCH_PLAN_ONLY"):  # tests: the rank layout, before any GPU call
        print(json.dumps({"rank": rank, "world": world, "gpus": a.gpus, "backend": a.dist_backend}), flush=True)
        return
    if a.dry_run:
        return dry_run(a, rank, world)
    W, H, B = a.width, a.height, a.batch
    params = disflow.preset_params(disflow.Preset[a.preset.upper()], W, H)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:  # before any GPU call (plain forks)
        affinity = len(os.sched_getaffinity(0))
        workers = a.cpu_workers or min(CPU_WORKER_CAP, affinity)
        c = cpu_baseline(params, W, H, a.cpu_seconds, workers)
        lib = os.path.basename(oracle_lib_for_baseline())
        cpu = {"value": c["value"], "unit": "frame-pairs/s", "cores": c["cores"], "kind": "port",
               "sample": f"{c['pairs']} synthetic {W}x{H} pairs, preset={a.preset}, in {c['cores']} host "
                         f"processes (one pair at a time each, like the reference) for {2 * a.cpu_seconds / 3:.0f} s, "
                         f"inputs generated before the clock ({min(c['cores'], 16)} seeded pairs, cycled); "
                         f"C oracle (oracle/dis_oracle.c as {lib}, gcc -O3 -ffp-contract=off)",
               "host": {"nproc": os.cpu_count(), "affinity_cpus": affinity, "physical_cores": physical_cores(),
                        "cpu_model": cpu_model(), "worker_cap": CPU_WORKER_CAP,
                        "note": f"measured on {workers} worker processes = min({CPU_WORKER_CAP}, affinity CPUs). "
                                "The affinity mask shows the whole host, but the GPU pool's operating rules "
                                f"allot one GPU's share, {CPU_WORKER_CAP} CPUs, to this job and ask worker pools "
                                "to be sized to it; the whole host (shared with the other GPUs' jobs) is not "
                                "measured. whole_host_estimate scales the measured per-process rate to the "
                                "physical cores: an extrapolation, not a measurement"},
               "single_core": {"value": c["single_core"]["value"], "pairs": c["single_core"]["pairs"],
                               "cores": 1},
               "per_process": c["value"] / c["cores"]}
        pc = physical_cores()
        if pc:
            cpu["whole_host_estimate"] = {"value": c["value"] / c["cores"] * pc, "cores": pc, "measured": False,
                                          "basis": f"per-process rate at {c['cores']} workers x {pc} physical cores "
                                                   "(no SMT gain, no memory-bandwidth loss assumed)"}
    if a.dist_backend != "nccl":  # gloo rehearsal: several ranks may share one GPU
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # read-only sclk / socket-power samples of this rank's GPU (amdgpu hwmon)
    # during the timed region and the roofline pass: a VALU-bound kernel's time
    # follows the clock, which follows the power cap
    from disflow import boxstate
    sampler = boxstate.Sampler(boxstate.torch_hwmon_dir(local))
    if world > 1:
        import torch.distributed as dist
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.dist_backend)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    wl = disflow.workload(params, W, H)

    seeds = [rank * B + k for k in range(B)]
    I0, I1 = make_pairs(seeds, W, H)
    d0 = torch.from_numpy(I0).to(dev)
    d1 = torch.from_numpy(I1).to(dev)
    out = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
    eng = disflow.DenseInverseSearch(params, W, H, max_batch=B, device=local)
    if a.streams:
        eng.set_concurrency(a.streams)
    # the calls go to a dedicated stream: HIP's null (default) stream carries
    # implicit synchronisation with the device's other streams (measured: the
    # two-context pattern below lost 7 % on it)
    stream = torch.cuda.current_stream(dev) if a.default_stream else torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)  # inputs uploaded on the default stream are complete

    def step():
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), stream.cuda_stream)

    # W warmup steps, then more untimed steps until WARMUP_FLOOR_S of GPU work
    # has run: at small W (the driver may pass --warmup 2) the card is still
    # ramping its clocks and a short timed region (K=5 is ~8 ms) reads low
    t_w = time.perf_counter()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    extra_warmup = 0
    while time.perf_counter() - t_w < a.warmup_floor:
        for _ in range(8):
            step()
        extra_warmup += 8
        torch.cuda.synchronize(dev)

    barrier()
    torch.cuda.synchronize(dev)
    with sampler.phase("timed"):
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        barrier()
        el = time.perf_counter() - t0

    # roofline pass (after the timed region): the same steps with the batch on
    # one stream, so the finest-level search launch runs without co-running
    # sub-batches; HIP dispatch events time every launch of it
    n_f, ms_f = 0, 0.0
    if not a.no_kernel_timing:
        eng.set_concurrency(1)
        step()
        eng.set_kernel_timing(True)  # (re)enabling starts a fresh measurement
        with sampler.phase("roofline"):
            for _ in range(max(10, a.steps // 5)):
                step()
            torch.cuda.synchronize(dev)
        n_f, ms_f = eng.kernel_time(disflow.KERNEL_SEARCH_FINEST)
        eng.set_kernel_timing(False)
        eng.set_concurrency(a.streams if a.streams else 2)
    # measured HBM peaks on this card (SURVEY 8d asks for a stream-copy peak
    # beside the 8 TB/s spec): device-to-device copy and fill of 1 GiB, events
    hbm_meas = None
    if rank == 0:
        nbytes = 1 << 30
        x = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
        y = torch.empty_like(x)
        x.fill_(1.0)

        def rate(fn, moved):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            e1.synchronize()
            return moved * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9

        hbm_meas = {"copy_GBps": rate(lambda: y.copy_(x), 2 * nbytes), "fill_GBps": rate(lambda: y.fill_(2.0), nbytes),
                    "note": "torch device copy (read+write bytes) and fill of 1 GiB, 10 reps"}
        del x, y
    # Serving pattern: two batches in flight -- steps issued
    # alternately to two contexts on two caller streams, one sub-batch stream
    # each, both replaying their graphs: no fork/join per call, and each
    # context's gap between calls is filled by the other's work. Same K steps
    # of B pairs, every flow written; reported beside `value` (which keeps one
    # batch at a time on one stream). (Linking the two contexts with
    # dis_pipeline_link forces eager enqueue: measured slower)
    piped = None
    if not a.no_pipelined:
        engs = [eng, disflow.DenseInverseSearch(params, W, H, max_batch=B, device=local)]
        strs = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]  # not the default stream (implicit syncs)
        out2 = torch.empty_like(out)
        outs2 = [out, out2]
        for e in engs:
            e.set_concurrency(1)

        def pstep(k):
            engs[k % 2].calc_device(B, d0.data_ptr(), d1.data_ptr(), outs2[k % 2].data_ptr(), strs[k % 2].cuda_stream)
        t_w = time.perf_counter()
        k = 0
        while k < max(2, a.warmup) or time.perf_counter() - t_w < a.warmup_floor:
            pstep(k)
            k += 1
            if k % 8 == 0:
                torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        for k in range(a.steps):
            pstep(k)
        torch.cuda.synchronize(dev)
        barrier()
        el_p = torch.tensor([time.perf_counter() - t2], dtype=torch.float64,
                            device=dev if a.dist_backend == "nccl" else "cpu")
        if world > 1:
            torch.distributed.all_reduce(el_p, op=torch.distributed.ReduceOp.MAX)
        same = bool(torch.equal(out2.view(torch.int32), out.view(torch.int32)))
        engs[1].close()
        del out2
        eng.set_concurrency(a.streams if a.streams else 2)
        piped = {"inflight": 2, "value": world * B * a.steps / float(el_p.item()), "unit": "frame-pairs/s",
                 "ms_per_step": float(el_p.item()) / a.steps * 1e3, "outputs_identical": same,
                 "note": "same K steps of B pairs per GPU, issued alternately to two contexts on two caller "
                         "streams (one sub-batch stream each, graphs replayed, no link); every flow computed "
                         "and written"}

    # DIS_PRECISION_FMA (opt-in tolerance mode): the same steps
    # timed the same way after the headline measurement, its finest launch
    # with dispatch events, and pair 0 against the oracle; reported in its own
    # sub-object -- `value` is always the bit-exact default path
    tol = None
    if not a.no_tolerance_mode:
        eng.set_precision(disflow.PRECISION_FMA)
        for _ in range(max(2, a.warmup // 2)):
            step()
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        barrier()
        el_f = torch.tensor([time.perf_counter() - t1], dtype=torch.float64,
                            device=dev if a.dist_backend == "nccl" else "cpu")
        if world > 1:
            torch.distributed.all_reduce(el_f, op=torch.distributed.ReduceOp.MAX)
        n_ff, ms_ff = 0, 0.0
        if not a.no_kernel_timing:
            eng.set_concurrency(1)
            step()
            eng.set_kernel_timing(True)
            for _ in range(max(10, a.steps // 5)):
                step()
            torch.cuda.synchronize(dev)
            n_ff, ms_ff = eng.kernel_time(disflow.KERNEL_SEARCH_FINEST)
            eng.set_kernel_timing(False)
            eng.set_concurrency(a.streams if a.streams else 2)
        fma_out0 = out[0].cpu().numpy()
        eng.set_precision(disflow.PRECISION_EXACT)
        step()  # leave `out` holding the exact path's flows (the gather and the parity check use it)
        torch.cuda.synchronize(dev)
        launch_ms_f = ms_ff / max(n_ff, 1)
        fl = B * wl["search_flops_finest"] / (launch_ms_f * 1e-3) / 1e12 if n_ff else None
        tol = {"precision": "fma (dis_set_precision(DIS_PRECISION_FMA))",
               "value": world * B * a.steps / float(el_f.item()), "unit": "frame-pairs/s",
               "ms_per_step": float(el_f.item()) / a.steps * 1e3,
               "finest_search": {"avg_launch_ms": launch_ms_f, "achieved": fl, "peak": FMA_PEAK_TFLOPS,
                                 "unit": "TFLOP/s", "frac": fl / FMA_PEAK_TFLOPS if fl else None,
                                 "note": "same algorithmic op count as the exact line; peak = vector f32 "
                                         "with FMA counted as 2 ops"},
               "stated_tolerance": "DESIGN.md 2 / profiles/tolerance_r02.json; GPU test tests/test_gpu_tolerance.py"}

    # max over ranks of the timed region (before the gather: the timing stands whatever it does)
    el_t = torch.tensor([el], dtype=torch.float64, device=dev if a.dist_backend == "nccl" else "cpu")
    if world > 1:
        torch.distributed.all_reduce(el_t, op=torch.distributed.ReduceOp.MAX)
    el = float(el_t.item())

    # the path's one collective, outside the timed region: the
    # last step's flows of every rank gathered to rank 0 over RCCL/xGMI
    gather = None
    if world > 1:
        barrier()
        torch.cuda.synchronize(dev)
        gather = gather_and_verify(out, B, rank, world, a.dist_backend, sync=lambda: torch.cuda.synchronize(dev))

    # parity spot check on rank 0: pair 0 of the last step vs the C oracle
    max_epe = None
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_binding
        exp = oracle_binding.calc_from_params(I0[0], I1[0], params)
        got = out[0].cpu().numpy()
        max_epe = float(np.sqrt(((got.astype(np.float64) - exp) ** 2).sum(-1)).max())
        if tol is not None:
            e = np.sqrt(((fma_out0.astype(np.float64) - exp) ** 2).sum(-1))
            tol["epe_vs_oracle_pair0"] = {"mean": float(e.mean()), "p99.9": float(np.percentile(e, 99.9)),
                                          "max": float(e.max())}



    # one finest-level search launch per step in the roofline pass (B pairs)
    avg_ms = ms_f / max(n_f, 1)
    launches_per_step = 1
    flops_per_launch = B * wl["search_flops_finest"] / launches_per_step
    bytes_per_launch = B * wl["search_bytes_finest"] / launches_per_step
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if n_f else None
    achieved_gbs = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if n_f else None
    traffic = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            if (tj.get("batch") == B and tj.get("width") == W and tj.get("preset") == a.preset
                    and tj.get("launches_per_step") in (None, launches_per_step)):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    sampler.close()
    box = {"hwmon": sampler.dir, "timed": sampler.summary("timed"), "roofline_pass": sampler.summary("roofline"),
           "note": "rank 0's GPU: sclk (hwmon freq1_input) and socket power (power1_input) sampled every ~2 ms, "
                   "read-only; the quoted peaks assume 2400 MHz"}
    clock = (box["roofline_pass"] or {}).get("sclk_MHz_mean")
    if rank == 0:
        pairs = world * B * a.steps
        line = {
            "metric": METRIC,
            "value": pairs / el,
            "unit": "frame-pairs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_extra": {"steps": extra_warmup, "floor_s": a.warmup_floor,
                             "note": "untimed steps added after the W warmup steps until the floor "
                                     "of warm-up time has elapsed (clock ramp)"},
            "ms_per_step": el / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded value-noise pairs warped by a smooth sinusoidal flow, dis_synth_pair)",
            "config": {"workload": f"{W}x{H} preset={a.preset}, {B} pairs/GPU/step, inputs+outputs in HBM",
                       "width": W, "height": H, "preset": a.preset, "global_batch": world * B,
                       "knobs": {"C": params.coarsest_scale, "F": params.finest_scale, "ps": params.patch_size,
                                 "it": params.iterations, "overlap": params.patch_overlap, "steps": wl["steps"]},
                       "parallelism": f"pairs sharded over {world} rank(s), no data-path collective"},
            "roofline": {"bound": "valu", "kernel": "k_search8, finest-level launch (patch inverse search)",
                         "achieved": achieved, "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": (achieved / VALU_PEAK_TFLOPS) if achieved else None, "traffic": traffic,
                         "avg_launch_ms": avg_ms, "launches": n_f,
                         "clock_MHz": clock,
                         "frac_at_clock": (achieved / (VALU_PEAK_TFLOPS * clock / 2400.0))
                         if (achieved and clock) else None,
                         "algorithmic_flops_per_launch": flops_per_launch,
                         "hbm": {"achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": (achieved_gbs / HBM_PEAK_GBS) if achieved_gbs else None,
                                 "algorithmic_bytes_per_launch": bytes_per_launch},
                         "note": "bound by f32 VALU issue (bit-exact reference rounding: no FMA); "
                                 "FLOPs = DESIGN.md 4 count x patches in the launch (all B pairs); "
                                 "duration = HIP dispatch events of the finest-level launch in a "
                                 "one-stream pass after the timed region; traffic = PMC HBM bytes per "
                                 "launch of that kernel (profiles/traffic.json); clock_MHz = mean sclk sampled "
                                 "during that pass, frac_at_clock = achieved / (peak x clock / 2400 MHz)"},
            "pipeline_hbm_frac": wl["algorithmic_bytes"] * pairs / el / 1e9 / HBM_PEAK_GBS,
            "hbm_measured_peak": hbm_meas,
            "box_state": box,
            "cpu_baseline": cpu,
            "gather": gather,
            "max_epe_vs_oracle": max_epe,
            "tolerance_mode": tol,
            "pipelined": piped,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
