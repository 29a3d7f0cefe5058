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
    value is the faster of the two in nodes/s; both are reported."""
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
    best = dict(max(runs.values(), key=lambda r: r["value"]))
    best["runs"] = runs
    return best


def share_rccl_id(rank, world, make_id):
    """Rank 0 creates the RCCL unique id and sends it to every other rank."""
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500")) + 17
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
    # the reference binary itself is unbuildable in this image (DESIGN.md
    # §2); BASELINE.md §2 holds its -t 1 run from the survey container
    rec["reference_t1_survey"] = {"wall_s": REF_PF08184_T1_S, "nodes_per_s": REF_PF08184_T1_NODES / REF_PF08184_T1_S,
                                  "source": "BASELINE.md §2 (msa_pastar -t 1, survey container)"}
    rec["ratio_nodes_per_s_vs_reference_t1"] = rate / (REF_PF08184_T1_NODES / REF_PF08184_T1_S)
    rec["target"] = ">= 10x the CPU reference's nodes/s (BASELINE.json north_star)"
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
    engine = Engine(seqs, device=device, n_shards=world, shard_rank=rank, rccl_id=rid)
    opt = PAStarOpt(batch_nodes=args.batch, table_slots_log2=args.table_log2,
                    pool_entries=args.pool, band=args.band, depth=args.depth, profile=True, mode=args.mode)

    def step():
        engine.init()
        r = engine.pa_star(opt)
        rows = engine.alignment()
        return r, rows

    # the first search on this context: its buffers, the graph capture and
    # the per-problem constants are set up inside it (untimed warmup)
    engine.synchronize()
    t_first = time.perf_counter()
    step()
    engine.synchronize()
    first_search = time.perf_counter() - t_first
    for _ in range(max(0, args.warmup - 1)):
        step()

    results = []
    engine.barrier()
    engine.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        results.append(step())
    engine.synchronize()
    engine.barrier()
    elapsed = time.perf_counter() - t0

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
                   "lengths": [len(s) for s in seqs.seqs], "hash": "FZORDER/12",
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
    print(json.dumps(line), flush=True)
    engine.barrier()
    engine.close()


if __name__ == "__main__":
    main()
