#!/usr/bin/env python3
"""Benchmark of the MI355X PAStar engine (BASELINE.json metric).

One *step* = one full search of the workload on the GPU(s): PairAlign
precompute (wavefront kernel), the batched device-resident A* to the optimal
SP score, and the backtrace of the alignment.  The sequences are synthetic
(tools/gen_synthetic.py) and uploaded before the timed
region; contexts and device buffers are created before it too.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

N > 1 runs one rank per GPU (launched by torch.distributed.run, which sets
RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT); the ranks shard one search by
the reference's z-order owner hash and exchange nodes over RCCL (strong
scaling: the total work is one search).  Rank 0 prints one JSON line.

The timed region is bracketed by a barrier and a device synchronize on both
sides and the time is the max over ranks, as the driver contract asks; both go
through the engine (RCCL allreduce, hipDeviceSynchronize) rather than
torch.distributed / torch.cuda: importing torch in this process would load
torch's bundled ROCm 7.0 HIP runtime in place of the system 7.2 one, under
which hipGraph capture of the step loop with event nodes is refused.  The
RCCL unique id is handed from rank 0 to the others over a TCP socket on
MASTER_PORT + 17.

Roofline: the expand kernel's average launch duration is measured live in the
timed region by the kernel itself (first-block start to last-block end on the
100 MHz device clock, accumulated on the device; PAStarOpt.profile), because
HIP event nodes inside the replayed graph cost several microseconds per step;
profiles/ holds the rocprofv3 kernel-trace summary of the same command for the
cross-check.
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "A* nodes expanded/sec + wall-clock to optimal SP alignment, 1/2/4/8 MI355X"
GOLDEN = os.path.join(ROOT, "tests", "golden")
WORKLOADS = {  # name -> (fasta fixture, BASELINE.json config it stands for, known optimal score)
    "syn4x200_s1": ("syn4x200_s1.fasta", "configs[1]: 4 synthetic seqs x200 residues", 149875),
    "PF08184": ("PF08184.fasta", "configs[2]: PF08184.fasta", 24450),
    "kinase": ("kinase.fasta", "configs[3]: kinase.fasta", 421546),
    "syn8x400_s5": ("syn8x400_s5.fasta", "configs[4]: 8 synthetic seqs x400 residues", 1318889),
    "syn8x100_s3": ("syn8x100_s3.fasta", "survey point: 8 synthetic seqs x100 residues", 703569),
}
# serial (-t 1) expansion counts of the reference, for the useful rate
SERIAL_EXPANSIONS = {"syn4x200_s1": 22089, "PF08184": 60, "kinase": 4497279}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E spec peak
# measured on one MI355X (tools/micro/atomic_rate.hip, profiles/r2_atomic_rate.txt):
# random 8-B loads over a 2 GB array, and random device-scope 8-B atomics
# (18.4 G/s over 2 GB, 27 G/s over 256 MB)
RANDOM_LOAD_PEAK_GS = 52.0
RANDOM_ATOMIC_PEAK_GS = 18.4
# the reference's own PF08184 run at -t 1: 60 expansions in
# about 0.11 s (its receiver's backoff sleeps floor the wall time)
REF_PF08184_T1_S, REF_PF08184_T1_NODES = 0.11, 60


def bytes_per_expansion(n):
    """Algorithmic HBM bytes of one expansion:
    B_exp = S + 16P + N + 2MS, S = 2N + 12 (parent record, 4 H cells per pair,
    residues, neighbour records written + one table probe each)."""
    s = 2 * n + 12
    p = n * (n - 1) // 2
    m = (1 << n) - 1
    return s + 16 * p + n + 2 * m * s


def env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def cpu_baseline(fasta, budget_s, known, legs=("t1", "tN")):
    """The oracle's PAStar restatements on the same input, on the host cores
    (-t 1 and -t $(nproc)): the serial search (1 core) and
    the multithreaded one (z-order owned lists per thread, inbox exchange;
    threads = the box's CPU share, at most 16), each repeated for about half
    of `budget_s` seconds (bounded sample, at least one search).  The line's
    value is the leg with the shorter wall time to the optimum; both are
    reported."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind  # test infrastructure: the CPU baseline leg only
    o = oracle_bind.Oracle(fasta=fasta)
    threads = env_int("PASTAR_CPU_THREADS", min(16, os.cpu_count() or 1))

    def sample(search, cores):
        runs, exp, secs = 0, 0, 0.0
        t_start = time.perf_counter()
        while True:
            r = search()
            if r["score"] != known:
                raise RuntimeError("CPU baseline score %d != %d" % (r["score"], known))
            runs += 1
            exp += r["expansions"]
            secs += r["seconds"]
            if time.perf_counter() - t_start >= budget_s / 2 or runs >= 10000:
                break
        return {"value": exp / secs, "unit": "nodes/s", "cores": cores, "kind": "port",
                "sample": "%d full %s searches of the workload (%d expansions each on average, %.2f s of search)"
                          % (runs, "serial" if cores == 1 else "%d-thread" % cores, exp // runs, secs),
                "wall_to_optimal_s": secs / runs, "score": r["score"]}

    runs = {}
    if "t1" in legs:
        runs["t1"] = sample(o.astar, 1)
    if "tN" in legs:
        runs["t%d" % threads] = sample(lambda: o.pastar_mt(threads), threads)
    # the line's baseline is the leg that reaches the optimum sooner (the
    # multithreaded search expands several times the serial count, so its
    # nodes/s can be higher while its search is slower)
    best = dict(min(runs.values(), key=lambda r: r["wall_to_optimal_s"]))
    best["chosen_by"] = "wall_to_optimal_s"
    best["runs"] = runs
    return best


def share_rccl_id(rank, world, make_id, offset=17):
    """Rank 0 creates the RCCL unique id and sends it to every other rank."""
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500")) + offset
    if rank == 0:
        rid = make_id()
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind(("", port))
        srv.listen(world)
        srv.settimeout(300)
        for _ in range(world - 1):
            conn, _ = srv.accept()
            conn.sendall(rid)
            conn.close()
        srv.close()
        return rid
    deadline = time.time() + 300
    while True:
        try:
            with socket.create_connection((addr, port), timeout=10) as c:
                buf = b""
                while len(buf) < 128:
                    chunk = c.recv(128 - len(buf))
                    if not chunk:
                        raise ConnectionError("short read")
                    buf += chunk
                return buf
        except OSError:
            if time.time() > deadline:
                raise
            time.sleep(0.2)


def pmc_summary(workload):
    """The committed rocprofv3 summary of the same workload
    (profiles/pmc_<workload>.json, tools/pmc_summary.py): HBM bytes per expand
    launch from the PMC passes, and the rocprof expand time per timed search
    of the traced bench command."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % workload)
    if not os.path.exists(path):
        return {}, None
    with open(path) as f:
        return json.load(f), os.path.relpath(path, ROOT)


def north_star(Engine, PAStarOpt, Sequences, device, searches=200, cpu_seconds=4.0):
    """BASELINE.json's target config: PF08184 at 1 GPU, wall to the optimal
    alignment (PairAlign + search + backtrace, one search per call) and
    expansions/s, next to the CPU ports on the same host cores and the
    reference's own -t 1 figure from the survey."""
    name, (fasta_name, _, known) = "PF08184", WORKLOADS["PF08184"]
    fasta = os.path.join(GOLDEN, fasta_name)
    seqs = Sequences.from_fasta(fasta)
    opt = PAStarOpt(profile=True)
    t_cold = time.perf_counter()
    eng = Engine(seqs, device=device)
    t_ctx = time.perf_counter()
    eng.init()
    r = eng.pa_star(opt)
    eng.alignment()
    cold = time.perf_counter() - t_ctx
    walls, exps, kern, loop = [], 0, 0.0, 0.0
    for _ in range(searches):
        t = time.perf_counter()
        eng.init()
        r = eng.pa_star(opt)
        eng.alignment()
        walls.append(time.perf_counter() - t)
        if r.score != known:
            raise RuntimeError("PF08184 score %d != %d" % (r.score, known))
        exps += r.expansions_all
        kern += r.expand_ms
        loop += r.seconds
    eng.close()
    walls.sort()
    wall = sum(walls) / len(walls)
    rate = exps / sum(walls)
    rec = {"workload": name, "baseline_config": WORKLOADS[name][1], "engine": "solo" if r.solo else "batched",
           "searches": searches, "score": r.score, "score_ok": r.score == known,
           "expansions_per_search": exps / searches, "wall_to_optimal_s": wall,
           "wall_to_optimal_s_median": walls[len(walls) // 2], "nodes_per_s": rate,
           "kernel_us_per_search": 1e3 * kern / searches, "launch_to_result_s": loop / searches,
           "cold_context_wall_to_optimal_s": cold, "context_create_s": t_ctx - t_cold}
    cpu = cpu_baseline(fasta, cpu_seconds, known)
    rec["cpu_port"] = cpu["runs"]
    for k, leg in cpu["runs"].items():
        rec["ratio_nodes_per_s_vs_port_%s" % k] = rate / leg["value"]
        rec["ratio_wall_vs_port_%s" % k] = leg["wall_to_optimal_s"] / wall
    # Throughput: K independent searches of the problem in one launch
    # (pastar_gpu_search_many, one workgroup each), timed at the C-ABI, next
    # to the host cores each running serial searches of the same problem.
    rec["many"] = many_throughput(Engine, Sequences, seqs, device, known, cpu["runs"]["t1"]["value"], fasta)
    # The target's ratio, stated plainly: against the CPU port timed on this
    # box (a CPU path that does the reference's work per expansion).  One
    # 60-expansion search is latency-bound on the GPU (59 dependent levels),
    # so its ratio is below 1; many searches per launch fill the chip.
    rec["ratio_vs_cpu_port_single_search"] = rec["ratio_nodes_per_s_vs_port_t1"]
    rec["ratio_vs_cpu_port_many_searches"] = rec["many"]["ratio_nodes_per_s_vs_port_t1"]
    # the reference binary itself is unbuildable in this image; BASELINE.md
    # §2 holds its -t 1 run from the survey container.  Its Phase-2 time is
    # floored by the receiver thread's backoff sleep (PAStarReceiver.cpp:
    # 30-35), so it is no measure of its search: listed, not compared.
    rec["reference_t1_survey"] = {"wall_s": REF_PF08184_T1_S, "nodes_per_s": REF_PF08184_T1_NODES / REF_PF08184_T1_S,
                                  "source": "BASELINE.md §2 (msa_pastar -t 1, survey container)",
                                  "comparable": False,
                                  "why": "sleep-floored Phase-2 time on another machine: an upper bound, not the search time"}
    rec["target"] = ">= 10x the CPU reference's nodes/s (BASELINE.json north_star)"
    return rec


def many_throughput(Engine, Sequences, seqs, device, known, port_t1_rate, fasta, k=1024, reps=30, cpu_seconds=3.0):
    """K contexts of one problem searched in one launch, repeated; the C-ABI
    call is timed (ctypes), the Python result objects are not built."""
    import ctypes
    import threading
    from mpi_pastar_msa_amd import _native as nat
    engines = [Engine(seqs, device=device).init() for _ in range(k)]
    try:
        arr = (ctypes.c_void_p * k)(*[e._ctx.value for e in engines])
        out = (nat.pastar_result * k)()
        fn = nat.lib().pastar_gpu_search_many
        for _ in range(3):
            nat.check(fn(arr, k, None, out))
        t0 = time.perf_counter()
        for _ in range(reps):
            rc = fn(arr, k, None, out)
        dt = (time.perf_counter() - t0) / reps
        nat.check(rc)
        if any(r.score != known for r in out):
            raise RuntimeError("search_many: wrong score")
        exp = sum(r.expansions_all for r in out)
        rows = engines[k // 2].alignment()
    finally:
        for e in engines:
            e.close()
    rec = {"searches_per_launch": k, "launches": reps, "seconds_per_launch": dt, "nodes_per_s": exp / dt,
           "searches_per_s": k / dt, "score_ok": True, "alignment_cols": len(rows[0]),
           "ratio_nodes_per_s_vs_port_t1": exp / dt / port_t1_rate}
    # the host's cores each running serial searches of the same problem
    # (threads over the oracle's C search: the call releases the GIL)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind
    threads = env_int("PASTAR_CPU_THREADS", min(16, os.cpu_count() or 1))
    counts, csecs = [0] * threads, [0.0] * threads
    stop = time.perf_counter() + cpu_seconds
    oracles = [oracle_bind.Oracle(fasta=fasta) for _ in range(threads)]

    def work(i):
        while time.perf_counter() < stop:
            r = oracles[i].astar()
            counts[i] += r["expansions"]
            csecs[i] += r["seconds"]

    ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    # every core's own rate inside the C search (the interpreter's time
    # between calls is not charged to the CPU), summed over the cores
    cpu_rate = sum(c / t for c, t in zip(counts, csecs) if t > 0)
    rec["cpu_port_independent_searches"] = {"value": cpu_rate, "unit": "nodes/s", "cores": threads, "kind": "port",
                                            "sample": "%d threads, each repeating the serial search for %.0f s"
                                                      % (threads, cpu_seconds)}
    rec["ratio_nodes_per_s_vs_port_all_cores"] = exp / dt / cpu_rate
    return rec


def sharded_shift(n, world):
    """The z-order partition's shift (msa_pastar -s) this bench runs with: the
    reference's default 12 on one GPU; across GPUs, cells of 8 positions a
    coordinate for N <= 6 (shift 18: fewer owner changes along a path, so the
    shards' block-local chains reach further per step: kinase at 8 shards 262
    -> 127 steps, 16 M -> 6 M records) and the default for wider fan-outs
    (syn8x400 at 8 shards expands 6.6 M nodes at 12, 10.7 M at 18).  Measured
    with the in-process shard group on one GPU (tools/gpu/probe_shards.py)."""
    if world <= 1:
        return 12
    return 18 if n <= 6 else 12


def measure(engine, opt, steps, warmup):
    """`warmup` untimed searches (the first sets up the context's buffers,
    graph capture and per-problem constants), then `steps` timed ones
    between barriers and device synchronizes.  Returns (results, elapsed,
    first_search)."""
    def step():
        engine.init()
        r = engine.pa_star(opt)
        rows = engine.alignment()
        return r, rows

    engine.synchronize()
    t_first = time.perf_counter()
    step()
    engine.synchronize()
    first_search = time.perf_counter() - t_first
    for _ in range(max(0, warmup - 1)):
        step()
    results = []
    engine.barrier()
    engine.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        results.append(step())
    engine.synchronize()
    engine.barrier()
    return results, time.perf_counter() - t0, first_search


def sub_record(name, Engine, PAStarOpt, Sequences, rccl_unique_id, rank, world, device, steps, warmup, port_offset,
               cpu_seconds, cpu_legs):
    """One more BASELINE config measured the same way as the headline
    workload (every rank takes part when world > 1): wall to the optimal
    alignment, nodes/s, the expand kernel's roofline fraction, and on one
    GPU the CPU port beside it (bounded sample)."""
    fasta_name, cfg_desc, known = WORKLOADS[name]
    fasta = os.path.join(GOLDEN, fasta_name)
    seqs = Sequences.from_fasta(fasta)
    n = len(seqs.seqs)
    rid = share_rccl_id(rank, world, rccl_unique_id, port_offset) if world > 1 else None
    shift = sharded_shift(n, world)
    eng = Engine(seqs, device=device, n_shards=world, shard_rank=rank, rccl_id=rid, hash_shift=shift)
    results, elapsed, first = measure(eng, PAStarOpt(profile=True), steps, warmup)
    exp_all = sum(r.expansions_all for r, _ in results)
    exp_local = sum(r.expansions for r, _ in results)
    kern_ms = sum(r.expand_ms for r, _ in results)
    launches = sum(r.expand_launches for r, _ in results)
    exchanged = sum(r.exchanged for r, _ in results)
    if world > 1:
        elapsed = eng.allreduce([int(elapsed * 1e9)], "max")[0] / 1e9
        exchanged = eng.allreduce([exchanged], "sum")[0]
    score = results[-1][0].score
    eng.close()
    if score != known:
        raise RuntimeError("%s: score %d != %d" % (name, score, known))
    wall = elapsed / steps
    b_exp = bytes_per_expansion(n)
    avg_launch_s = (kern_ms / 1e3) / max(launches, 1)
    achieved = (exp_local / max(launches, 1)) * b_exp / avg_launch_s / 1e9 if launches and kern_ms else 0.0
    rec = {"workload": name, "baseline_config": cfg_desc, "n_gpus": world, "hash": "FZORDER/%d" % shift,
           "searches": steps, "score": score, "score_ok": True, "wall_to_optimal_s": wall,
           "nodes_per_s": exp_all / elapsed, "expansions_per_search": exp_all / steps,
           "steps_per_search": sum(r.steps for r, _ in results) / len(results),
           "first_search_on_context_s": first,
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "kernel": "expand_kernel (rank 0)",
                        "bytes_per_expansion": b_exp, "avg_launch_us": avg_launch_s * 1e6, "launches": launches}}
    if name in SERIAL_EXPANSIONS:
        rec["useful_rate"] = SERIAL_EXPANSIONS[name] / wall
    if world > 1:
        rec["records_exchanged_per_search"] = exchanged / steps
        rec["host_waits_per_search"] = sum(r.host_waits for r, _ in results) / len(results)
    elif cpu_legs and rank == 0:
        rec["cpu_baseline"] = cpu_baseline(fasta, cpu_seconds, known, cpu_legs)
        rec["wall_ratio_vs_cpu"] = rec["cpu_baseline"]["wall_to_optimal_s"] / wall
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="syn4x200_s1", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="batch_nodes (0 = engine default)")
    ap.add_argument("--table-log2", type=int, default=0)
    ap.add_argument("--pool", type=int, default=0, help="open-list entry pool (0 = engine default)")
    ap.add_argument("--band", type=int, default=0, help="f band of one step (0 = engine default)")
    ap.add_argument("--depth", type=int, default=0, help="expansion levels per step (0 = engine default)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-legs", default="t1,tN",
                    help="CPU baseline legs: t1 (serial), tN (multithreaded); syn8x400's serial search takes minutes")
    ap.add_argument("--no-north-star", action="store_true", help="skip the PF08184 sub-record (N = 1 only)")
    ap.add_argument("--no-sub-records", action="store_true",
                    help="skip the kinase / syn8x400_s5 sub-records (BASELINE configs[3], [4]) of the default line")
    ap.add_argument("--hash-shift", type=int, default=-1, help="owner partition shift (-1 = the bench's choice)")
    ap.add_argument("--mode", default="auto", choices=["auto", "batched", "solo"], help="search engine")
    args = ap.parse_args()

    world = env_int("WORLD_SIZE", 1)
    rank = env_int("RANK", 0)
    local_rank = env_int("LOCAL_RANK", 0)
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("--gpus %d needs torch.distributed.run with %d processes" % (args.gpus, args.gpus))
        args.gpus = world

    from mpi_pastar_msa_amd import Engine, PAStarOpt, Sequences, rccl_unique_id

    dist_on = world > 1
    rid = share_rccl_id(rank, world, rccl_unique_id) if dist_on else None

    fasta_name, cfg_desc, known = WORKLOADS[args.workload]
    fasta = os.path.join(GOLDEN, fasta_name)
    seqs = Sequences.from_fasta(fasta)
    n = len(seqs.seqs)
    device = env_int("PASTAR_BENCH_DEVICE", local_rank)  # override for single-GPU rehearsals
    shift = args.hash_shift if args.hash_shift >= 0 else sharded_shift(n, world)
    engine = Engine(seqs, device=device, n_shards=world, shard_rank=rank, rccl_id=rid, hash_shift=shift)
    opt = PAStarOpt(batch_nodes=args.batch, table_slots_log2=args.table_log2,
                    pool_entries=args.pool, band=args.band, depth=args.depth, profile=True, mode=args.mode)

    results, elapsed, first_search = measure(engine, opt, args.steps, args.warmup)

    exp_all = sum(r.expansions_all for r, _ in results)
    exp_local = sum(r.expansions for r, _ in results)
    kern_ms = sum(r.expand_ms for r, _ in results)
    select_ms = sum(r.select_ms for r, _ in results)
    gap_ms = sum(r.gap_ms for r, _ in results)
    launches = sum(r.expand_launches for r, _ in results)
    loop_s = sum(r.seconds for r, _ in results) / len(results)
    score = results[-1][0].score
    if dist_on:  # max over ranks (ns resolution)
        mx = engine.allreduce([int(elapsed * 1e9), int(loop_s * 1e9), int(first_search * 1e9)], "max")
        elapsed, loop_s, first_search = mx[0] / 1e9, mx[1] / 1e9, mx[2] / 1e9
    # wall to the optimal alignment: a whole step (PairAlign, search,
    # backtrace; inputs resident), as the metric names it
    wall = elapsed / args.steps
    # BASELINE configs[3] and [4] beside the headline workload, measured the
    # same way at this world size (collective: every rank takes part)
    subs = {}
    if args.workload == "syn4x200_s1" and not args.no_sub_records:
        for k, (name, st, wu, secs, legs) in enumerate([("kinase", 5, 2, 4.0, ("tN",)),
                                                        ("syn8x400_s5", 3, 1, 20.0, ("tN",))]):
            subs[name] = sub_record(name, Engine, PAStarOpt, Sequences, rccl_unique_id, rank, world, device, st, wu,
                                    18 + k, secs, None if args.no_cpu_baseline else legs)
    # the roofline is reported for rank 0's expand kernel
    if rank != 0:
        engine.barrier()
        engine.close()
        return

    value = exp_all / elapsed
    b_exp = bytes_per_expansion(n)
    avg_launch_s = (kern_ms / 1e3) / max(launches, 1)
    achieved = (exp_local / max(launches, 1)) * b_exp / avg_launch_s / 1e9 if launches else 0.0
    pmc, traffic_src = pmc_summary(args.workload)
    traffic = pmc.get("hbm_bytes_per_launch")
    alg_per_launch = (exp_local / max(launches, 1)) * b_exp if launches else 0.0
    exp_per_search = exp_local / args.steps
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": "solo_kernel" if results[-1][0].solo else "expand_kernel", "bytes_per_expansion": b_exp,
            "avg_launch_us": avg_launch_s * 1e6, "launches": launches,
            "avg_select_tail_us": 1e3 * select_ms / max(launches, 1),
            "avg_gap_us": 1e3 * gap_ms / max(launches, 1),
            "traffic_source": traffic_src}
    if traffic and alg_per_launch:
        # PMC bytes over algorithmic bytes per launch (> 1: re-reads and
        # partial lines; the PMC read side is an upper bound, see the source)
        roof["traffic_ratio"] = traffic / alg_per_launch
    gen = sum(r.generated for r, _ in results)
    if gen and exp_local and launches and not results[-1][0].solo:
        # the same fraction with the children the kernel did relax in place of the reference's 2^N - 1 per
        # expansion (partial expansion for N >= 7 leaves most of them ungenerated; border nodes have fewer)
        # (capped at 2^N - 1: the dive also relaxes the children of nodes whose expansion did not count)
        s_rec = 2 * n + 12
        kids = min(gen / exp_local, float((1 << n) - 1))
        b_rel = s_rec + 16 * (n * (n - 1) // 2) + n + 2 * kids * s_rec
        roof["children_relaxed_per_expansion"] = kids
        roof["frac_children_relaxed"] = (exp_local / launches) * b_rel / avg_launch_s / 1e9 / HBM_PEAK_GBS
    if kern_ms > 0 and gen and not results[-1][0].solo:
        # the random-access view of the same kernel: every generated child
        # probes its node-table slot (one random line read; at most one
        # device-scope atomic), against the chip's measured random-load rate
        rate = gen / (kern_ms / 1e3) / 1e9
        roof["probes"] = {"achieved": rate, "peak": RANDOM_LOAD_PEAK_GS, "unit": "G probes/s",
                          "frac": rate / RANDOM_LOAD_PEAK_GS, "atomic_peak": RANDOM_ATOMIC_PEAK_GS,
                          "children_per_search": gen / args.steps, "source": "profiles/r2_atomic_rate.txt"}
    us_search = pmc.get("rocprof_expand_us_per_search_timed")
    if us_search:
        # the same algorithmic bytes per search over the expand time per
        # search that rocprofv3 measured for this workload's bench command
        # (profiles/, regenerated at the commit named there)
        roof["frac_rocprof"] = exp_per_search * b_exp / (us_search * 1e-6) / 1e9 / HBM_PEAK_GBS
        roof["rocprof_expand_us_per_search"] = us_search
        roof["rocprof_commit"] = pmc.get("commit")
        roof["rocprof_cmd"] = pmc.get("cmd")
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "nodes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (tools/gen_synthetic.py, SURVEY.md §8(d)-gen)" if args.workload.startswith("syn")
                else "reference fixture %s" % fasta_name,
        "config": {"workload": args.workload, "baseline_config": cfg_desc, "n_seqs": n,
                   "lengths": [len(s) for s in seqs.seqs], "hash": "FZORDER/%d" % shift,
                   "batch_nodes": args.batch or (262144 if n <= 6 else 65536), "depth": args.depth or (128 if n <= 4 else 8),
                   "parallelism": "shard%d" % world},
        "score": score,
        "score_ok": score == known,
        "wall_to_optimal_s": wall,
        "search_loop_s": loop_s,
        "first_search_on_context_s": first_search,
        "first_over_warm": first_search / wall,
        "expansions_per_search": exp_all / args.steps,
        "steps_per_search": sum(r.steps for r, _ in results) / len(results),
        "engine": "solo" if results[-1][0].solo else "batched",
        "graph_replay": bool(results[-1][0].graph_replay),
        "roofline": roof,
    }
    if args.workload in SERIAL_EXPANSIONS:
        line["useful_rate"] = SERIAL_EXPANSIONS[args.workload] / wall
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(fasta, args.cpu_seconds, known, tuple(args.cpu_legs.split(",")))
    if world == 1 and not args.no_north_star and args.workload != "PF08184":
        line["north_star"] = north_star(Engine, PAStarOpt, Sequences, device)
    if subs:
        line["sub_records"] = subs
    if world > 1:
        line["records_exchanged_per_search"] = sum(r.exchanged for r, _ in results) / len(results)
        line["host_waits_per_search"] = sum(r.host_waits for r, _ in results) / len(results)
    print(json.dumps(line), flush=True)
    engine.barrier()
    engine.close()


if __name__ == "__main__":
    main()
