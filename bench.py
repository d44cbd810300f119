#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): in-pod bf16 matmul TFLOPS at 1/2/4/8 MI355X
(+ notebook cold-start p50 from the native control plane when requested).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched by
``torch.distributed.run`` with one rank per GPU (RCCL). Run directly with ``--gpus N > 1`` (no
WORLD_SIZE in the env) it launches the N ranks itself (kubeflow_rm_amd.parallel.launch.run_ranks:
child processes started before this process touches the GPU, private rendezvous port, one failing
rank stops the rest and fails the run). Each rank is one notebook pod's GPU running
the K1 readiness op: a bf16 GEMM C = A @ B^T (8192^3 by default) on the hand-written gfx950 MFMA
kernel. A "step" = one such GEMM on every GPU. ``--prewarm-s`` (default 1 s) of untimed GEMMs settle
the GPU clock, then W untimed warmup steps, then exactly K timed steps bracketed by barrier + device
sync on both sides; the slowest rank's time is used. After the timed region rank 0 times
torch.matmul (hipBLASLt) on the same operands (``torch_matmul_tflops_per_gpu``, never the value). ``value`` is
the whole-job aggregate TFLOPS (N x per-GEMM FLOPs / max-rank time). Weak scaling: per-GPU work
is fixed as N grows. Data: synthetic uniform [-1, 1) bf16 operands (random data, not zeros:
zero operands inflate MFMA clocks — cdna_hip_programming.md §5.4 rule 25).

Cold start (rank 0, after the timed region, while the other ranks wait on a CPU-side barrier with
their GPU memory released): ``--coldstart-runs`` (default 10) Notebook CREATE -> Ready runs of ONE
notebook requesting all N GPUs, through the native control plane (process pods: no container
runtime), with the in-pod readiness op on the allocated GPUs (N >= 2: one-shot peer all-reduce over
xGMI). Reported with p50 / p90 and the per-phase p50 breakdown; the same for the ODH OAuth spawn path,
the torch-ready server (imports torch + runs a GEMM before Ready) and that server forked from the
kubelet's pre-imported interpreter (``--pod-zygote``). Then the control-plane latencies of
BASELINE configs 3 and 5 (Profile with GPU quota ready; TensorBoard and PVCViewer ready) on the same
native control plane, and configs 4 and 5 as stated (``config4_*`` / ``config5_*``): one Notebook
holding all N GPUs runs the RCCL all-reduce smoke inside its pod (``--rccl``; ``--rccl-single`` at
N = 1), then a TensorBoard and a PVCViewer attach to that notebook's RWO workspace PVC and are
co-scheduled onto its node.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_START = time.time()
METRIC = "notebook pod cold-start p50 (s) + in-pod bf16 matmul TFLOPS at 1/2/4/8 MI355X"


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--prewarm-s", type=float, default=float(os.environ.get("KFAMD_BENCH_PREWARM_S", "1.0")),
                   help="untimed GEMM time before the W warmup steps, so the timed steps run at the "
                        "sustained clock rather than on the DVFS ramp from idle (0 disables)")
    # --gemm-m/-n/-k: the spellings to use behind torch.distributed.run, whose parser rejects "--m"
    # as an ambiguous prefix of its own options even after the script name
    p.add_argument("--m", "--gemm-m", dest="m", type=int, default=8192)
    p.add_argument("--n", "--gemm-n", dest="n", type=int, default=8192)
    p.add_argument("--k", "--gemm-k", dest="k", type=int, default=8192)
    p.add_argument("--coldstart-runs", type=int, default=int(os.environ.get("KFAMD_COLDSTART_RUNS", "10")),
                   help="cold-start runs of one N-GPU notebook through the native control plane (rank 0)")
    p.add_argument("--coldstart-torch-runs", type=int, default=int(os.environ.get("KFAMD_COLDSTART_TORCH_RUNS", "5")),
                   help="cold-start runs with the torch-ready notebook server (torch import + GEMM before Ready)")
    p.add_argument("--compare-torch", action=argparse.BooleanOptionalAction, default=True,
                   help="also time torch.matmul (hipBLASLt) on the same operands, after the timed region "
                        "(rank 0; reported as torch_matmul_tflops_per_gpu, never as the value)")
    p.add_argument("--no-allreduce-sweep", action="store_true",
                   help="skip the RCCL all-reduce busbw sweep run after the timed region when N > 1")
    p.add_argument("--force-dist", action=argparse.BooleanOptionalAction,
                   default=os.environ.get("KFAMD_FORCE_DIST", "") not in ("", "0"),
                   help="run the multi-GPU code path at WORLD_SIZE=1 too: RCCL process group, gloo CPU group, "
                        "barriers, the RCCL / peer all-reduce sweeps and the cold-start parking "
                        "(e.g. torchrun --nproc-per-node 1 bench.py --force-dist on a one-GPU box)")
    p.add_argument("--ab-blocks", type=int, default=5,
                   help="interleaved blocks of STEPS GEMMs, ours then torch.matmul (hipBLASLt), after the timed "
                        "region: both medians and their ratio are reported (0 disables)")
    p.add_argument("--budget-s", type=float, default=float(os.environ.get("KFAMD_BENCH_BUDGET_S", "450")),
                   help="wall-clock budget from process start for everything after the timed region: extras "
                        "that do not fit are reported as skipped, one that hangs as timeout (bench_extras.py)")
    return p.parse_args()


COLD_START_NOTE = ("process pods (no container runtime). cold_start_* = the product's default path: the "
                   "jupyter-pytorch-rocm notebook server (imports torch, runs a GEMM on its GPU before Ready) forked "
                   "from the kubelet's pre-imported interpreter (--pod-zygote, on by default), a 1-GPU pod taking "
                   "the zygote's warm child of its GPU (HIP + device context already up); cold_start_stub_* = a "
                   "server that imports nothing (control plane + readiness op alone); cold_start_torch_ready_fresh_* "
                   "= the torch server in a fresh interpreter (--pod-zygote=false); cold_start_odh_* = ODH path with "
                   "the OAuth proxy + reconciliation lock. The GPU readiness op runs as a native sidecar overlapping "
                   "the server start. *_failures = runs not Ready within the per-run timeout, with pod diagnostics "
                   "in cold_start_failure_diagnostics")


def _cs_keys(prefix: str, cs: dict) -> dict:
    out = {f"{prefix}_runs": len(cs["runs"]), f"{prefix}_p50_s": cs["p50_s"], f"{prefix}_p90_s": cs["p90_s"],
           f"{prefix}_phases_p50_s": cs.get("phases_p50_s"), f"{prefix}_failures": len(cs.get("failures") or [])}
    if cs.get("server_warmup_p50_ms"):
        out[f"{prefix}_server_p50_ms"] = cs["server_warmup_p50_ms"]
    if cs.get("warm_children") is not None:
        out[f"{prefix}_warm_children"] = cs["warm_children"]
    if cs.get("truncated"):
        out[f"{prefix}_truncated"] = True
    if cs.get("failures"):
        # (not "<prefix>_failures": for the default path that is the count's own key)
        out.setdefault("cold_start_failure_diagnostics", {})[prefix] = cs["failures"]
    return out


def run_cold_starts(ex, args, world: int) -> None:
    """Rank 0: the cold-start variants and the control-plane latencies, each its own extra."""
    from kubeflow_rm_amd.bench_coldstart import measure_cold_start, measure_control_plane, measure_gpu_notebook_configs

    def merge_failures(e, out):
        f = out.pop("cold_start_failure_diagnostics", None)
        if f:
            e.data.setdefault("cold_start_failure_diagnostics", {}).update(f)
        return out

    def default_path(e):
        # the product's default: torch-ready server, kubelet --pod-zygote (kflite's default), warm GPU child
        cs = measure_cold_start(runs=args.coldstart_runs, gpus_per_notebook=world, server="torch-ready",
                                namespace="bench", zygote=True, timeout=30, deadline=e.deadline())
        out = _cs_keys("cold_start", cs)
        out.update({"cold_start_gpus_per_notebook": world, "cold_start_readiness": cs.get("readiness"),
                    "cold_start_note": COLD_START_NOTE})
        # BASELINE §3 north-star #2: controller reconcile latency, from the control plane's own
        # controller_runtime_reconcile_time_seconds histogram over these runs
        nbr = (cs.get("reconcile") or {}).get("notebook-controller") or {}
        out["reconcile_p50_ms"] = (nbr.get("reconcile") or {}).get("p50_ms")
        out["reconcile_p99_ms"] = (nbr.get("reconcile") or {}).get("p99_ms")
        out["reconcile_queue_p50_ms"] = (nbr.get("queue") or {}).get("p50_ms")
        out["reconcile_by_controller"] = cs.get("reconcile")
        return out

    ex.run("cold_start", lambda e: merge_failures(e, default_path(e)), est_s=20, timeout_s=150)
    # the control plane + readiness op alone (a server that imports nothing)
    ex.run("cold_start_stub", lambda e: merge_failures(e, _cs_keys("cold_start_stub", measure_cold_start(
        runs=args.coldstart_runs, gpus_per_notebook=world, namespace="bench-stub", timeout=30,
        deadline=e.deadline()))), est_s=10, timeout_s=90)
    if args.coldstart_torch_runs > 0:
        # the torch-ready server in a fresh interpreter (--pod-zygote=false)
        ex.run("cold_start_torch_ready_fresh", lambda e: merge_failures(e, _cs_keys(
            "cold_start_torch_ready_fresh", measure_cold_start(
                runs=args.coldstart_torch_runs, gpus_per_notebook=world, server="torch-ready", namespace="bench-torch",
                timeout=30, deadline=e.deadline()))), est_s=15, timeout_s=120)
    # the fork's own spawn path: ODH webhook lock + OAuth proxy + two reconciles
    ex.run("cold_start_odh", lambda e: merge_failures(e, _cs_keys("cold_start_odh", measure_cold_start(
        runs=max(3, args.coldstart_runs // 2), gpus_per_notebook=world, odh_oauth=True, namespace="bench-odh",
        timeout=30, deadline=e.deadline()))), est_s=25, timeout_s=90)
    # BASELINE configs 3 and 5: Profile with GPU quota, TensorBoard + PVCViewer on a PVC
    ex.run("control_plane", lambda e: {"control_plane": measure_control_plane(runs=5)}, est_s=5, timeout_s=60)
    # BASELINE configs 4 and 5 as stated: one notebook holding all N GPUs runs the RCCL all-reduce
    # smoke in its pod (config4_*), then a TensorBoard and a PVCViewer attach to its RWO workspace
    # PVC and are co-scheduled onto its node (config5_*)
    ex.run("gpu_notebook_configs", lambda e: measure_gpu_notebook_configs(
        gpus_per_notebook=world, timeout=max(10.0, min(90.0, e.deadline() - time.time()))), est_s=10, timeout_s=120)


def self_launch(args) -> int:
    """``--gpus N`` without a launcher: run N ranks of this script (or of the JSON argv in
    KFAMD_BENCH_RANK_ARGV — the CPU test's stub worker) and return the job's exit code."""
    from kubeflow_rm_amd.parallel.launch import run_ranks
    argv = json.loads(os.environ.get("KFAMD_BENCH_RANK_ARGV") or "null") or \
        [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    return run_ranks(argv, args.gpus, master_addr="127.0.0.1")


def main() -> int:
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world} (n_gpus reports WORLD_SIZE)", file=sys.stderr)
    # the multi-GPU code path: world > 1, or forced at world 1 so one GPU executes it end to end
    distributed = world > 1 or args.force_dist
    if args.force_dist:
        os.environ["KFAMD_FORCE_DIST"] = "1"  # parallel.tp / parallel.dp follow the same switch
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and not os.environ.get("MASTER_PORT"):
            from kubeflow_rm_amd.parallel.dist import _free_port
            os.environ["MASTER_PORT"] = str(_free_port())
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        dist.init_process_group("nccl", device_id=dev)

    from kubeflow_rm_amd import ops

    M, N, K = args.m, args.n, args.k
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    a = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

    # correctness check of this very configuration against a fp32 reference: one row in every
    # 256-row macro-tile (a different row offset in each) against ALL N columns, so every output tile
    # of the XCD-remapped grid — and every wave's row range within the tiles — is compared
    ops.gemm_nt(a, b, out=c)
    rows = torch.tensor([t * 256 + (t * 37) % min(256, M - t * 256) for t in range((M + 255) // 256)], device=dev)
    ref = a.index_select(0, rows).float() @ b.float().t()
    err = (c.index_select(0, rows).float() - ref).abs().max().item()
    ok = err <= 1e-2 * ref.abs().max().item() + 1e-2

    def step():
        ops.gemm_nt(a, b, out=c)

    # DVFS: an idle MI355X needs a few hundred ms of load to settle its GFX clock; without this a
    # short K measures the ramp (20 steps = 16 ms), not the kernel
    t_pre = time.perf_counter()
    while time.perf_counter() - t_pre < args.prewarm_s:
        for _ in range(10):
            step()
        torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        step()

    def barrier():
        if distributed:
            dist.barrier(device_ids=[local_rank])

    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    dt = time.perf_counter() - t0

    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt_max = t.item()
    ms_per_step = dt_max / args.steps * 1e3
    flops = ops.flops(M, N, K)
    per_gpu_tflops = flops / (ms_per_step * 1e-3) / 1e12
    value = per_gpu_tflops * world

    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "TFLOPS (bf16 GEMM, aggregate over GPUs)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "prewarm_s": args.prewarm_s,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (uniform [-1,1) bf16 operands, random-init)",
        "config": {
            "model": f"in-pod bf16 matmul HIP smoke (K1 readiness op), C=A@B^T {M}x{N}x{K}",
            "global_batch": world,
            "seq_len": None,
            "parallelism": f"dp{world}",
        },
        "dist_path": "rccl" if distributed else "none",
        "per_gpu_tflops": round(per_gpu_tflops, 2),
        "kernel": "kfamd gemm_w4 (4 waves x 128x128, one wave/SIMD, asm MFMA 16x16x32 bf16 with AGPR accumulators, buffer_load..lds into a 5-slot LDS ring with the K loop unrolled over its 5-tile period, XCD remap, in-kernel edge tiles)",
        "check_rows": int(rows.numel()),
        "correct": bool(ok),
        "max_abs_err_vs_fp32": err,
    }

    # everything after the timed region is an extra: own try, own deadline, overall budget, and a
    # watchdog that prints the line with what was measured if one of them hangs (bench_extras.py)
    from kubeflow_rm_amd.bench_extras import Extras, print_line
    import datetime
    # the CPU group's own timeout bounds every wait on it (ranks != 0 park on it during rank 0's
    # cold starts): past the budget a barrier raises instead of waiting for the 30-minute default
    cpu_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=args.budget_s + 60)) \
        if distributed else None

    def agree(flag: bool) -> bool:
        if not distributed:
            return flag
        f = torch.tensor([1 if flag else 0], dtype=torch.int32)
        dist.all_reduce(f, op=dist.ReduceOp.MIN, group=cpu_group)
        return bool(f.item())

    ex = Extras(args.budget_s, t_start=T_START, rank=rank, agree=agree,
                emit=lambda rep: print_line({**line, **rep}))

    if args.compare_torch and args.ab_blocks > 0 and rank == 0:
        # fair comparison with hipBLASLt: interleaved ABAB blocks of STEPS GEMMs
        # on the same operands and the same warm part, not one torch block after ours
        def ab(_ex):
            import statistics
            ours, theirs = [], []

            def block(fn):
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                for _ in range(args.steps):
                    fn()
                torch.cuda.synchronize(dev)
                return flops * args.steps / (time.perf_counter() - t1) / 1e12

            def torch_mm():
                torch.matmul(a, b.t(), out=c)

            for _ in range(3):
                torch_mm()
            for _ in range(args.ab_blocks):
                ours.append(block(step))
                theirs.append(block(torch_mm))
            mo, mt = statistics.median(ours), statistics.median(theirs)
            return {"ab_ours_tflops_median": round(mo, 1), "ab_hipblaslt_tflops_median": round(mt, 1),
                    "ab_ratio_ours_over_hipblaslt": round(mo / mt, 4), "ab_blocks": args.ab_blocks,
                    "ab_ours_tflops": [round(x, 1) for x in ours], "ab_hipblaslt_tflops": [round(x, 1) for x in theirs],
                    "torch_matmul_tflops_per_gpu": round(mt, 1)}
        ex.run("gemm_ab_vs_hipblaslt", ab, est_s=3, timeout_s=60)

    if distributed and not args.no_allreduce_sweep:
        # BASELINE §3 "RCCL all-reduce busbw over xGMI" on the same N GPUs, outside the timed GEMM
        # region (every rank participates; rank 0 reports)
        # 8 B .. 1 GiB, fp32 and bf16, algbw and busbw = algbw * 2(n-1)/n
        def rccl(_ex):
            from kubeflow_rm_amd.parallel.collectives import allreduce_sweep
            out = {}
            for name, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
                sw = allreduce_sweep(max_bytes=1 << 30, min_bytes=8, step=8, iters_small=20, iters_large=5,
                                     dtype=dt, device=dev)
                out[f"rccl_allreduce_{name}"] = [{"bytes": r["bytes"], "us": round(r["us"], 1),
                                                  "algbw_GBps": round(r["algbw_GBps"], 1),
                                                  "busbw_GBps": round(r["busbw_GBps"], 1)} for r in sw]
                torch.cuda.empty_cache()
            return out
        ex.run("rccl_allreduce", rccl, est_s=20, timeout_s=90, collective=True)

        # the hand-written peer all-reduces (K3) on the same GPUs, and the per-link xGMI ceiling
        # their busbw is judged against (153 GB/s x 7 links per GPU, spec)
        def peer(_ex):
            from kubeflow_rm_amd.parallel.collectives import fast_allreduce_sweep
            return {"allreduce_oneshot_bf16": fast_allreduce_sweep([16 << s for s in range(0, 15, 2)], "oneshot"),
                    "allreduce_twoshot_bf16": fast_allreduce_sweep([256 << 10 << s for s in range(0, 9, 2)], "twoshot")}
        ex.run("peer_allreduce", peer, est_s=15, timeout_s=60, collective=True)

        def xgmi(_ex):
            from kubeflow_rm_amd.parallel.collectives import xgmi_probe
            torch.cuda.empty_cache()
            xg = xgmi_probe()
            return {"xgmi_peer": xg, "xgmi_peer_GBps": xg["pair_GBps_median"]}
        ex.run("xgmi_probe", xgmi, est_s=10, timeout_s=60, collective=True)

    if args.coldstart_runs > 0:
        # the N-GPU notebook needs every GPU: free this rank's memory, park ranks != 0 on a CPU
        # (gloo) barrier — an RCCL barrier would keep a spinning kernel on their GPUs
        del a, b, c
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        if distributed:
            dist.barrier(group=cpu_group)
        if rank == 0:
            run_cold_starts(ex, args, world)
        if distributed:
            # ranks != 0 wait here for rank 0's cold starts: the CPU group's timeout (budget + 60 s)
            # bounds the wait, and a rank that times out fails the run
            try:
                dist.barrier(group=cpu_group)
            except Exception as e:  # noqa: BLE001
                print(f"rank {rank}: cold-start barrier failed: {type(e).__name__}: {e}", file=sys.stderr)
                ex.finish()
                if rank == 0:
                    ex.emit_once({"rank_barrier_error": f"{type(e).__name__}: {e}"[:500]})
                sys.stdout.flush()
                os._exit(124)

    line.update(ex.finish())
    if rank == 0:
        ex.emit_once()
    if distributed:
        dist.destroy_process_group()
    if not ok:
        return 1
    return 124 if ex.timed_out else 0


if __name__ == "__main__":
    sys.exit(main())
