#!/usr/bin/env python3
"""bench.py -- CoCoA+ on the BASELINE.json headline workload (config C2: an
rcv1-shaped synthetic SVM, n = 677,399 rows, d = 47,236 features, ~75.6 nnz
per row, lambda = 1e-4, K = 64 partitions, H = n/K local steps), on N MI355X.

One "step" = one CoCoA+ round (64 local SDCA solvers per GPU x H coordinate
steps, deltaW fold, RCCL all-reduce when N > 1, w update) followed by the
duality-gap / test-error evaluation (so the gap trajectory is measured inside
the timed region).  value = coordinate updates per second over all GPUs.

Scaling (cocoa_amd.configs): weak by default -- every GPU holds its own
677,399-row shard of one seeded problem (64 partitions each, K = 64*N
globally, H unchanged); --scaling strong keeps one fixed problem (n, K) and
splits its partitions over the GPUs (C3: K = 64 on 1-8 GPUs; C4: K = 1,024).

Prints one JSON line (rank 0).  N > 1 ranks, one process per GPU, either way:
  python bench.py --gpus N      (this process spawns the N ranks itself, before
                                 any GPU call, and relays rank 0's line)
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
A rank whose WORLD_SIZE differs from --gpus fails.
"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CoCoA+ SVM wall-clock to duality gap 1e-4; coord updates/s at 1/2/4/8 GPUs"
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak


from cocoa_amd.configs import CONFIGS  # noqa: E402  (BASELINE.json configs)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def solver_bytes_per_round(tr, H, seed_t, method="cocoa+", solver="gram"):
    """Algorithmic bytes of one solver launch (DESIGN.md
    section 3 table), per coordinate step of a sampled row with z entries:
      sparse SDCA (gram / chain): 16 (row_ptr pair) + 8 (y) + 16 (alpha r/w)
        + 36 z (12 B CSR entry + w gather + deltaW gather + deltaW write) for
        CoCoA+ / MbCD, 44 z for CoCoA (its task-local w is read and written too);
      dense rows (dense solver): 8 d (the row) + 20 (sample, y, ||x||^2) -- w and
        deltaW stay in registers, no gathers;
      mb-SGD: 16 + 8 + 20 z (entry + w gather); local SGD: 16 + 8 + 36 z."""
    import cocoa_amd
    K = tr.num_parts
    if solver == "dense":
        return K * H * (8 * tr.num_features + 20)
    z = np.diff(tr.row_ptr)
    per_step, per_entry = {"cocoa+": (40, 36), "mbcd": (40, 36), "cocoa": (40, 44),
                           "mbsgd": (24, 20), "localsgd": (24, 36)}[method]
    tot = 0
    for k in range(K):
        p0, p1 = int(tr.part_ptr[k]), int(tr.part_ptr[k + 1])
        idx = cocoa_amd.jrandom_ints(seed_t, p1 - p0, H)
        tot += per_step * H + per_entry * int(z[p0 + idx].sum())
    return tot


def eval_bytes(tr, te, d, dense):
    """Algorithmic bytes of one evaluation pass (OptUtils.scala:57-98): every
    train and test entry once, y, alpha, w; CSR rows 12 B per entry plus the row
    pointers, dense rows (X[n][d], no column indices) 8 B per entry."""
    if dense:
        return 8 * tr.n * d + 8 * tr.n + 8 * tr.n + 8 * d + 8 * te.n * d + 8 * te.n
    return (12 * tr.nnz + 8 * (tr.n + 1) + 8 * tr.n + 8 * tr.n + 8 * d
            + 12 * te.nnz + 8 * (te.n + 1) + 8 * te.n)


def comm_mismatch(requested, rank, world, comm):
    """The error message when the library's communicator (cocoa_comm_info) is not
    the exchange this run asked for, else None.  An N-rank run must run its deltaW
    all-reduce over exactly the requested transport with all N ranks: a
    multi-GPU line that quietly ran over another transport (or fewer ranks) is not
    a measurement of the path north_star names (CoCoA.scala:45-48 over xGMI)."""
    if world <= 1:
        return None
    if comm is None or comm.get("world") != world or comm.get("rank") != rank:
        return f"bench.py: rank {rank}/{world} but the library's communicator says {comm}"
    if comm.get("transport") != requested:
        return (f"bench.py: --transport {requested} requested with {world} ranks but the library's communicator "
                f"runs {comm.get('transport')}: refusing to report a line over another exchange")
    return None


def num(v):
    """v as a float when it is a number (amdsmi returns "N/A" strings for fields a
    box does not expose), else None."""
    return float(v) if isinstance(v, (int, float)) and not isinstance(v, bool) else None


class GpuTelemetry:
    """Clocks, power and temperature of this rank's GPU (amdsmi), so that runs on
    different boxes can be told apart from regressions: snap() reads the current
    gfx (sclk), memory (mclk) and fabric (fclk) clocks, socket power, the power
    cap and the hotspot / memory temperatures; start()/stop() sample every 20 ms
    on a thread for the timed region.  Every read is best effort (a field is None
    where the box does not expose it)."""

    def __init__(self, bus_id=None, domain_id=None):
        self.h = None
        self.samples = []
        self._thr = None
        self._stop = False
        try:
            import amdsmi
            self.smi = amdsmi
            amdsmi.amdsmi_init()
            hs = amdsmi.amdsmi_get_processor_handles()
            for h in hs:
                try:
                    bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
                    dom, bus = int(bdf.split(":")[0], 16), int(bdf.split(":")[1], 16)
                    if bus_id is None or (bus == bus_id and (domain_id is None or dom == domain_id)):
                        self.h, self.bdf = h, bdf
                        break
                except Exception:
                    continue
        except Exception as e:  # no amdsmi / no permission: telemetry stays empty
            self.err = repr(e)

    def _try(self, f):
        try:
            return f()
        except Exception:
            return None

    def snap(self):
        try:
            return self._snap()
        except Exception as e:
            return {"error": repr(e)}

    def _snap(self):
        if self.h is None:
            return None
        smi, h = self.smi, self.h
        clk = lambda t: num(self._try(lambda: smi.amdsmi_get_clock_info(h, t)["clk"]))  # noqa: E731
        pw = self._try(lambda: smi.amdsmi_get_power_info(h)) or {}
        cap = self._try(lambda: smi.amdsmi_get_power_cap_info(h)) or {}
        temp = lambda t: num(self._try(lambda: smi.amdsmi_get_temp_metric(  # noqa: E731
            h, t, smi.AmdSmiTemperatureMetric.CURRENT)))
        gm = self._try(lambda: smi.amdsmi_get_gpu_metrics_info(h)) or {}
        pick = lambda v: num(v) if num(v) not in (0xFFFF, 0xFFFFFFFF) else None  # noqa: E731
        return {"t": time.time(),
                "sclk_mhz": clk(smi.AmdSmiClkType.SYS), "mclk_mhz": clk(smi.AmdSmiClkType.MEM),
                "fclk_mhz": clk(smi.AmdSmiClkType.DF),
                "avg_gfxclk_mhz": pick(gm.get("average_gfxclk_frequency")),
                "power_w": pick(pw.get("current_socket_power")) or pick(pw.get("average_socket_power")),
                "power_cap_w": (num(cap.get("power_cap")) / 1e6) if num(cap.get("power_cap")) is not None else None,
                "temp_hotspot_c": temp(smi.AmdSmiTemperatureType.HOTSPOT),
                "temp_mem_c": temp(smi.AmdSmiTemperatureType.VRAM)}

    def start(self):
        if self.h is None:
            return
        import threading
        self.samples, self._stop = [], False

        def run():
            while not self._stop:
                s = self.snap()
                if s:
                    self.samples.append(s)
                time.sleep(0.02)
        self._thr = threading.Thread(target=run, daemon=True)
        self._thr.start()

    def stop(self):
        if self._thr is not None:
            self._stop = True
            self._thr.join(timeout=2)
            self._thr = None
        return self.summary()

    def summary(self):
        try:
            return self._summary()
        except Exception as e:  # telemetry never fails the bench
            return {"error": repr(e)}

    def _summary(self):
        s = self.samples
        if not s:
            return None
        out = {"samples": len(s)}
        for k in ("sclk_mhz", "mclk_mhz", "fclk_mhz", "avg_gfxclk_mhz", "power_w", "temp_hotspot_c"):
            v = [x[k] for x in s if isinstance(x.get(k), (int, float))]
            if v:
                out[k] = {"min": min(v), "mean": sum(v) / len(v), "max": max(v)}
        return out


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, timeout_s=None):
    """Launch n ranks of this script (one process per GPU, CoCoA.scala:45-48's
    partition blocks), each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
    and relay rank 0's stdout.  Runs in a parent that has made no GPU call (no
    torch.cuda, no Engine), so the children own the devices.  Returns the worst
    child exit status; once one rank fails the others get 30 s to end (they
    would wait at a barrier forever) and are then killed by PID."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env, cwd=ROOT,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=r == 0))
    chunks = []
    import threading
    drain = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    drain.start()
    t0 = time.time()
    first_fail = None
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad and first_fail is None:
            first_fail = time.time()
        late = (first_fail is not None and time.time() - first_fail > 30) or \
               (timeout_s is not None and time.time() - t0 > timeout_s)
        if late:
            for p in procs:
                if p.poll() is None:
                    log(f"killing rank pid {p.pid}")
                    p.send_signal(signal.SIGKILL)
        time.sleep(0.2)
    drain.join(timeout=10)
    sys.stdout.write("".join(chunks))
    sys.stdout.flush()
    rcs = [p.returncode for p in procs]
    log(f"ranks exited with {rcs}")
    return max((abs(rc) for rc in rcs), default=0) if any(rcs) else 0


def main():
    if "RANK" not in os.environ and "WORLD_SIZE" not in os.environ:
        ap0 = argparse.ArgumentParser(add_help=False)
        ap0.add_argument("--gpus", type=int, default=1)
        a0, _ = ap0.parse_known_args()
        if a0.gpus > 1:
            sys.exit(spawn_ranks(a0.gpus, sys.argv[1:]))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="BASELINE.json config (c2 = the headline line; c3/c4 are extra measurement lines)")
    ap.add_argument("--method", default="cocoa+", choices=["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"],
                    help="C5 five-method comparison: the method whose rounds are timed")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: every GPU holds its own n-row shard (K = parts*N); strong: one fixed problem "
                         "(n rows, K = parts) whose partitions are split over the GPUs")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "host"],
                    help="rank exchange inside libcocoa_hip.so: RCCL over xGMI (one GPU per rank) or HOST (TCP)")
    ap.add_argument("--solver", default="auto", choices=["auto", "gram", "chain", "dense"],
                    help="fast-mode SDCA local solver (cocoa_set_solver)")
    # (20 warmup rounds, ~40 ms: the amdsmi telemetry showed the gfx clock still
    # ramping 1.9 -> 2.1 GHz through a 3-round warmup's timed region)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--strict", action="store_true", help="bit-exact mode (default: fast)")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--d", type=int, default=None)
    ap.add_argument("--nnz", type=float, default=None)
    ap.add_argument("--parts", type=int, default=None)
    ap.add_argument("--lam", type=float, default=None)
    ap.add_argument("--n-test", type=int, default=None)
    ap.add_argument("--gap-target", type=float, default=1e-4)
    ap.add_argument("--gap-max-rounds", type=int, default=400)
    ap.add_argument("--cpu-seconds", type=float, default=30.0,
                    help="bound on the CPU baseline's fresh run to the gap target")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gap", action="store_true")
    ap.add_argument("--stats-kernels", default="solver",
                    help="kernels bracketed with HIP events in the timed region (default: the dominant kernel "
                         "the roofline reads; each bracketed launch adds two event packets to the step, "
                         "solver,eval: 7.8 us more per C2 step, profiles/r06/ab_r10g_events.txt)")
    ap.add_argument("--stats-all", action="store_true",
                    help="HIP events around every kernel in the timed region (default: the solver and the eval only)")
    ap.add_argument("--eval-sync", action="store_true",
                    help="read each round's evaluation back before enqueuing the next round (cocoa_eval) instead "
                         "of the default deferred read-back (cocoa_eval_begin / _end)")
    ap.add_argument("--pipeline", action="store_true",
                    help="evaluate each round beside the next one (cocoa_eval_async, the next round's x.w from "
                         "xw_produce_kernel) instead of in line; measured slower on C2 (3.01-3.04 vs 2.90 ms: "
                         "the side work then outgrows the solver)")
    ap.add_argument("--launch-probe", action="store_true",
                    help="launcher check (no GPU): rank 0 prints {rank, world, master} and every rank exits")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    for k in ("n", "d", "nnz", "parts", "lam", "n_test"):
        if getattr(args, k) is None:
            setattr(args, k, cfg[k])
    sdca = args.method in ("cocoa+", "cocoa", "mbcd")  # methods with a dual (alpha) and so a duality gap
    if not sdca:
        args.no_gap = True

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch N ranks as "
                         f"'bench.py --gpus N' (spawns them) or torch.distributed.run --nproc-per-node N")
    if args.launch_probe:
        if rank == 0:
            print(json.dumps({"rank": rank, "world": world, "local_rank": local_rank, "transport": args.transport,
                              "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}))
        return
    import torch
    import torch.distributed as dist
    if world > 1:
        # control plane only (communicator id, barriers, max over ranks): the
        # deltaW / objective exchange runs inside libcocoa_hip.so over RCCL
        dist.init_process_group("gloo")

    import cocoa_amd  # noqa: F401
    from cocoa_amd import Engine, configs
    from cocoa_amd.dist import DistributedCoCoA

    # ---- data: this rank's share of the seeded problem (cocoa_amd.configs) ----
    t0 = time.time()
    sh = configs.share(args.config, rank=rank, world=world, scaling=args.scaling, n=args.n, d=args.d, nnz=args.nnz,
                       parts=args.parts, lam=args.lam, n_test=args.n_test,
                       threads=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))
    tr, te = sh.train, sh.test
    K_glob, n_glob, H = sh.k_glob, sh.n_glob, sh.H
    log(f"rank {rank}: data n={tr.n} nnz={tr.nnz} d={args.d} K_loc={tr.num_parts} K={K_glob} H={H} "
        f"gen {time.time() - t0:.1f}s")

    # one GPU per rank; ranks beyond the visible devices share them (HOST
    # transport rehearsals on a one-GPU box -- RCCL needs distinct GPUs)
    ndev = max(torch.cuda.device_count(), 1)
    eng = Engine(device=local_rank % ndev, strict=args.strict)
    eng.set_train(tr, part_begin=sh.part_begin, num_parts_global=K_glob)
    eng.set_solver(args.solver)
    eng.set_test(te)
    eng.init(args.method, n_glob, 1 << 30, H, args.lam)
    runner = DistributedCoCoA(eng, transport=args.transport)
    comm = eng.comm_info()  # cocoa_comm_info: the exchange the library itself runs
    bad = comm_mismatch(args.transport, rank, world, comm)
    if bad:
        raise SystemExit(bad)

    def barrier():
        eng.sync()  # the engine's own HIP stream
        if world > 1:
            dist.barrier()
        eng.sync()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ---- warmup + timed steps ----------------------------------------------
    # Each round's evaluation in line behind it on the engine's stream, read back
    # once round t+1 is enqueued too (cocoa_eval_begin / _end; --eval-sync: read
    # back first, cocoa_eval), or with --pipeline (one device, fast mode) beside
    # the next round (cocoa_eval_async); every evaluation completes inside the
    # timed region.
    pipe = world == 1 and not args.strict and args.pipeline
    defer = not pipe and not args.eval_sync
    key = "gap" if sdca else "primal"

    def steps(t, count, stop=None):
        """count rounds from t, each evaluated; returns (values, rounds, t_next).
        stop(value) -> True ends the loop at the first round whose value satisfies it.
        Default: round t's evaluation is enqueued behind it (cocoa_eval_begin)
        and read back (cocoa_eval_end) once round t+1 is queued too, so the GPU
        never idles while the host reads a gap: 2.895-2.900 against 2.920-2.926
        ms per C2 step with --eval-sync (cocoa_eval after every round; r04p, one
        box).  (Round t+2's Gram rows wait for round t+1's plan: enqueued while
        the evaluation still ran, they took the CUs the next solver's workgroups
        need whole, 3.40 ms per step in r04f.)"""
        vals, rounds, pending = [], [], None
        for _ in range(count):
            runner.round(t)
            if pipe:
                if pending is not None:
                    vals.append(eng.eval_wait()[key])
                    rounds.append(pending)
                    if stop and stop(vals[-1]):  # (round t is still running; nothing pending)
                        return vals, rounds, t + 1
                eng.eval_async()
                pending = t
            elif defer:
                if pending is not None:
                    vals.append(runner.eval_end()[key])
                    rounds.append(pending)
                    pending = None
                    if stop and stop(vals[-1]):  # (round t is queued behind it; not evaluated)
                        return vals, rounds, t + 1
                runner.eval_begin()
                pending = t
            else:
                vals.append(runner.eval()[key])
                rounds.append(t)
                if stop and stop(vals[-1]):
                    return vals, rounds, t + 1
            t += 1
        if pending is not None:
            vals.append(eng.eval_wait()[key] if pipe else runner.eval_end()[key])
            rounds.append(pending)
        return vals, rounds, t

    props = torch.cuda.get_device_properties(local_rank % ndev) if torch.cuda.is_available() else None
    tele = GpuTelemetry(getattr(props, "pci_bus_id", None), getattr(props, "pci_domain_id", None))
    tele_before = tele.snap()

    t = 1
    _, _, t = steps(t, args.warmup)
    eng.stats_reset()
    # events only around the kernel the roofline reads (--stats-kernels): every
    # bracketed launch adds two event packets and ~4-5 us of launch latency each;
    # the evaluation's own roofline then reads the 5 launches after the timed region
    if not args.stats_all and hasattr(cocoa_amd._capi.lib(), "cocoa_stats_kernels"):
        eng.stats_kernels(args.stats_kernels.split(","))
    eng.stats_enable(True)
    barrier()
    tele_start = tele.snap()
    tele.start()
    ts = time.perf_counter()
    gaps, timed_rounds, t = steps(t, args.steps)
    barrier()
    dt = max_over_ranks(time.perf_counter() - ts)
    tele_timed = tele.stop()
    tele_end = tele.snap()
    stats = eng.kernel_stats()
    # the eval pass alone (in the timed loop it overlaps the next round's solver)
    eng.stats_reset()
    if not args.stats_all and hasattr(cocoa_amd._capi.lib(), "cocoa_stats_kernels"):
        eng.stats_kernels(["eval"])
    eng.sync()
    for _ in range(5):
        runner.eval()
    eval_alone = eng.kernel_stats().get("eval", {})
    eng.stats_enable(False)
    updates = K_glob * H * args.steps
    value = updates / dt
    log(f"timed {args.steps} rounds in {dt:.3f}s -> {value:.4g} updates/s; kernels {stats}")

    # ---- wall-clock to duality gap <= target (fresh run) -------------------
    ttg = None
    rounds_to_gap = None
    final_gap = None
    gap_run_s = None
    if not args.no_gap:
        eng.init(args.method, n_glob, 1 << 30, H, args.lam)
        barrier()
        tg = time.perf_counter()
        # the clock stops when the host knows a round's gap is <= target (pipelined:
        # while the round after it is already running)
        vals, rounds, _ = steps(1, args.gap_max_rounds, stop=lambda g: g <= args.gap_target)
        ttg = time.perf_counter() - tg
        barrier()
        ttg = max_over_ranks(ttg)
        final_gap = vals[-1]
        rounds_to_gap = rounds[-1] if final_gap <= args.gap_target else None
        log(f"gap {final_gap:.3g} after {rounds[-1]} rounds, {ttg:.3f}s")
        gap_run_s = ttg
        if rounds_to_gap is None:  # the target was not reached: no time-to-gap (gap_run_s says how long it ran)
            ttg = None

    # ---- roofline of the dominant kernel (solver) and of the eval pass -----
    plan = eng.plan()
    solver_ms = stats["solver"]["total_ms"] / max(stats["solver"]["launches"], 1)
    b_solver = np.mean([solver_bytes_per_round(tr, H, t_ + 0, args.method, plan.get("solver", "gram"))
                        for t_ in timed_rounds[:4]])
    ach = b_solver / (solver_ms * 1e-3) / 1e9
    # HBM traffic per launch from the committed PMC passes, only for the kernels
    # this run launched (fast mode, the C2 headline workload the passes profiled)
    traffic = traffic_eval = None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tf) and not args.strict and args.config == "c2" and args.method == "cocoa+" and world == 1:
        try:
            tk = json.load(open(tf)).get("kernels", {})
            rec = tk.get("solver_" + plan.get("solver", ""))
            traffic = rec["hbm_bytes_per_launch"] if rec else None
            # the evaluation's passes: the cold pass (eval_stream_kernel) and, with the
            # hot / cold split, the hot pass before it
            rec = tk.get("eval")
            traffic_eval = rec["hbm_bytes_per_launch"] if rec else None
            if traffic_eval is not None and plan.get("eval_split") and tk.get("eval_hot"):
                traffic_eval += tk["eval_hot"]["hbm_bytes_per_launch"]
        except Exception:
            traffic = traffic_eval = None
    # the eval's launch average over the timed region (HIP events on the
    # engine's stream); the 5 launches after it, with nothing beside them, are
    # reported as alone_ms
    eval_alone_ms = (eval_alone.get("total_ms", 0.0) / max(eval_alone.get("launches", 0), 1)) if eval_alone else None
    eval_in_line = stats.get("eval", {}).get("launches", 0) > 0  # (--stats-kernels without eval: alone only)
    eval_ms = stats["eval"]["total_ms"] / stats["eval"]["launches"] if eval_in_line else eval_alone_ms
    b_eval = eval_bytes(tr, te, args.d, plan.get("solver") == "dense")
    ach_eval = b_eval / (eval_ms * 1e-3) / 1e9

    # ---- CPU baseline: the oracle on this box's host cores (rank 0, N=1) ---
    # SURVEY.md 8(d) / BASELINE.md: the reference's Spark local[N] shape
    # (hingeDriver.scala:22) with N = min(K, hardware_concurrency) threads, one
    # task per partition, ordered serial deltaW reduce (CoCoA.scala:39-56), the
    # partition-parallel evaluation of OptUtils.scala:65-98 every round; a fresh
    # run to the same gap target as the GPU line, bounded by --cpu-seconds.
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle
        ncpu = os.cpu_count() or 1
        try:
            naff = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            naff = ncpu
        od = oracle.Data(tr.row_ptr, tr.col, tr.val, tr.y, tr.part_ptr, tr.num_features)
        ot = oracle.Data(te.row_ptr, te.col, te.val, te.y, te.part_ptr, te.num_features)

        def cpu_run(cores):
            run = oracle.Run(od, args.method, n_glob, H, args.lam, nthreads=cores)
            run.set_global_parts(K_glob)
            t_round = t_eval = 0.0
            rounds = 0
            cpu_gap = cpu_ttg = None
            tc0 = time.perf_counter()
            for r in range(1, args.gap_max_rounds + 1):
                tc = time.perf_counter()
                run.round(r)
                t_round += time.perf_counter() - tc
                rounds = r
                if sdca:
                    tc = time.perf_counter()
                    cpu_gap = run.eval(ot)["gap"]
                    t_eval += time.perf_counter() - tc
                    if not args.no_gap and cpu_gap <= args.gap_target:
                        cpu_ttg = time.perf_counter() - tc0
                        break
                if time.perf_counter() - tc0 > args.cpu_seconds:
                    break
            return {"value": tr.num_parts * H * rounds / max(t_round, 1e-9), "cores": cores,
                    "ms_per_round": t_round / rounds * 1e3, "eval_ms": (t_eval / rounds * 1e3) if sdca else None,
                    "time_to_gap_s": cpu_ttg, "rounds": rounds, "final_gap": cpu_gap,
                    "stopped_s": time.perf_counter() - tc0}

        cores = max(1, min(tr.num_parts, ncpu))
        c = cpu_run(cores)
        # the one-GPU job's fair share of a shared 8-GPU host's cores (16 on the
        # GPU boxes, where os.cpu_count() reports the whole machine)
        fair = cpu_run(min(16, cores)) if cores > 16 else None
        cpu = {"value": c["value"], "unit": "coord updates/s", "cores": cores, "cpu_count": ncpu, "affinity_cpus": naff,
               "kind": "port", "ms_per_round": c["ms_per_round"], "eval_ms": c["eval_ms"],
               "time_to_gap_s": c["time_to_gap_s"], "rounds": c["rounds"], "final_gap": c["final_gap"],
               "fair_share_16": fair,
               "sample": f"fresh {args.method} run of the same {args.config.upper()} shard (K={tr.num_parts}, H={H}) by the strict C "
                         f"oracle (oracle/cocoa_oracle.c) as Spark local[{cores}]: {cores} threads, one task per partition, "
                         f"ordered reduce, gap/test-error evaluation every round; {c['rounds']} rounds, "
                         + (f"gap {args.gap_target:g} reached in {c['time_to_gap_s']:.2f}s" if c["time_to_gap_s"] is not None
                            else f"stopped after {c['stopped_s']:.1f}s (--cpu-seconds) at gap {c['final_gap']}")
                         + ("; fair_share_16: the same run on 16 threads (a one-GPU job's share of the host)"
                            if fair else "")}
        log(f"cpu baseline {cpu}")

    if rank == 0:
        out = {
            "metric": METRIC, "value": value, "unit": "coord updates/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": args.scaling,
            # BASELINE.md publishes no number; its CPU-baseline plan
            # makes the measured local[N] oracle the baseline: coord updates/s ratio
            # BASELINE.md publishes no number for this metric: vs_baseline stays null;
            # the ratio to the CPU baseline measured here is reported on its own
            "vs_baseline": None,
            "vs_cpu_baseline": (value / cpu["value"]) if cpu else None,
            "time_to_gap_vs_cpu": (cpu["time_to_gap_s"] / ttg) if (cpu and ttg and cpu.get("time_to_gap_s")) else None,
            "time_to_gap_vs_cpu16": (cpu["fair_share_16"]["time_to_gap_s"] / ttg)
            if (cpu and ttg and cpu.get("fair_share_16") and cpu["fair_share_16"].get("time_to_gap_s")) else None,
            "dtype": "f64",
            "data": cfg["data"],
            "config": {"workload": f"{args.config.upper()} {cfg['shape']} {args.method} (n={tr.n}/GPU of {n_glob}, d={args.d}, "
                                   f"~{args.nnz} nnz/row, lambda={args.lam}, K={K_glob} ({tr.num_parts}/GPU), H=n/K={H}), "
                                   f"step = round + {'gap' if sdca else 'primal'} eval",
                       "method": args.method,
                       "n_total": n_glob, "K_total": K_glob, "H": H, "nnz_per_gpu": tr.nnz, "test_rows_per_gpu": te.n,
                       "mode": "strict" if args.strict else "fast",
                       "eval_flow": "pipelined (cocoa_eval_async)" if pipe else
                                    "deferred read-back (cocoa_eval_begin/_end)" if defer else "synchronous (cocoa_eval)",
                       "parallelism": f"dp{world}: {tr.num_parts} partitions per GPU, deltaW "
                                      f"{'all-reduce' if not args.strict else 'ordered chain'} inside libcocoa_hip.so "
                                      f"({args.transport.upper()})"},
            "time_to_gap_s": ttg, "rounds_to_gap": rounds_to_gap, "gap_target": args.gap_target,
            "gap_run_s": gap_run_s, "gap_max_rounds": args.gap_max_rounds,
            "final_gap": final_gap, "gap_trajectory_timed": gaps,
            "roofline": {"kernel": "solver (local SDCA, CoCoA.localSDCA)", "bound": "hbm", "achieved": ach,
                         "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS, "traffic": traffic,
                         "bytes_per_launch": b_solver, "avg_launch_ms": solver_ms,
                         "note": "latency-bound sequential chain (H dependent steps per partition)"},
            "roofline_eval": {"kernel": "eval (primal/dual/gap/test error SpMV)", "bound": "hbm", "achieved": ach_eval,
                              "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach_eval / PEAK_HBM_GBS,
                              "traffic": traffic_eval, "bytes_per_launch": b_eval, "avg_launch_ms": eval_ms,
                              "alone_ms": eval_alone_ms,
                              "note": ("avg_launch_ms: alone_ms (no events on the evaluation in the timed region, "
                                       "--stats-kernels)" if not eval_in_line else "avg_launch_ms: HIP events over the timed rounds (" +
                                      ("beside the next round's solver and Gram rows, --pipeline)" if pipe else
                                       "in line on the engine's stream; the next Gram rows wait for the next plan)"))
                                      + "; alone_ms: 5 launches after the timed region with nothing beside them"},
            "kernel_ms": {k: (v["total_ms"] / v["launches"]) for k, v in stats.items() if v["launches"] > 0},
            "cpu_baseline": cpu,
            "plan": plan,
            "comm": {"transport": comm["transport"] if world > 1 else None, "world": comm["world"] if world > 1 else 1},
            # the box's clocks / power / temperature (amdsmi): before warmup, at both
            # ends of the timed region and sampled every 20 ms inside it
            "gpu_telemetry": {"bdf": getattr(tele, "bdf", None), "before_warmup": tele_before,
                              "timed_start": tele_start, "timed_end": tele_end, "timed_samples": tele_timed,
                              "error": getattr(tele, "err", None)},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
