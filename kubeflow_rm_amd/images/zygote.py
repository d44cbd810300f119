"""Pre-imported interpreter ("zygote") for process pods: the node runtime's answer to the torch-ready
cold start, where ``import torch`` is 1.6-1.9 s of the 1.7-2.0 s (``profiles/r3_torch_import``).

The kubelet (``native/node/kubelet.cc``, ``--pod-zygote``) starts one zygote per image recipe that
names one, at node start. The zygote imports the recipe's preload modules (torch, the notebook
server) ONCE and then forks a fresh process per container start: the container's Python code runs
in its own process, session, environment, working directory, CPU mask and log file, with the
imports already done. It is the process-pod analogue of a pre-pulled, pre-started image sandbox;
the GPU is never touched before the fork, so every container creates its own HIP context
(HIP_VISIBLE_DEVICES from its own env) exactly as a cold process would.

Protocol (one AF_UNIX stream connection per container start, JSON lines):

  kubelet -> zygote   {"argv": ["-m", "module", args...], "env": ["K=V", ...], "cwd": "...",
                       "log": "/path/container.log", "cpus": [0, 1, ...]}
  zygote  -> kubelet  {"pid": 1234}                 (or {"error": "..."} and close)
  zygote  -> kubelet  {"exit": 0, "signal": 0}      when the process ends, then close

The connection stays open for the life of the container: it is how the kubelet (which is not the
process's parent) learns the exit status.

Warm GPU children (``--warm-devices 0,1,...``, ``--warm-modules``): per node GPU, the zygote keeps one
forked child that has already brought up HIP, torch's device context, the first GPU operation and the
framework's GEMM code object on that device alone (ROCR_VISIBLE_DEVICES=<d>, HIP_VISIBLE_DEVICES=0,
exactly the env the device plugin gives a 1-GPU pod on <d>), and then waits. A 1-GPU container
request that names ``"warm_device": d``, runs a module of ``--warm-modules`` and whose HIP-relevant env
matches the warm child's takes it: the child becomes the container (same steps as a fresh fork) and
the zygote forks the next warm child for <d>. The ~200 ms of HIP + device bring-up then happen
before the pod exists instead of on its cold-start path. Warm children die with the zygote until
claimed; nothing of a tenant ever runs in one before it is claimed, and each is used once. The kubelet kills the process group (the child calls
setsid). Safety: the zygote refuses to serve if its preload opened the GPU driver (/dev/kfd): a
fork of a process with a live HIP context is undefined. It also refuses if the preload left any
native thread besides the main one: fork() copies only the calling thread, so a lock another thread
held at that moment (malloc arenas, a BLAS server queue, the HIP runtime) would stay locked forever in
every container. ``import numpy`` alone starts one OpenBLAS worker per CPU, so the zygote imports
with the BLAS / OpenMP pools pinned to one thread and each container sizes its pools afterwards
(OpenBLAS grows its pool on demand, OpenMP spawns on the first parallel region).

Reference: the reference has no process runtime (L0 is Kubernetes); the cold-start path it
exercises is notebook_controller.go Reconcile -> StatefulSet -> kubelet -> image ENTRYPOINT
(components/example-notebook-servers/jupyter/s6/services.d/jupyterlab/run), which this replaces.
"""
from __future__ import annotations

import argparse
import gc
import importlib
import json
import os
import runpy
import select
import selectors
import signal
import socket
import sys
import time
import traceback


def _gpu_driver_open() -> bool:
    """True when this process holds the KFD / DRM device open (HIP initialised)."""
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                tgt = os.readlink(f"/proc/self/fd/{fd}")
            except OSError:
                continue
            if tgt == "/dev/kfd" or tgt.startswith("/dev/dri/"):
                return True
    except OSError:
        pass
    return False


def _set_pdeathsig() -> None:
    """Exit with the kubelet (Linux PR_SET_PDEATHSIG); the forked containers clear it (fork does)."""
    try:
        import ctypes
        libc = ctypes.CDLL(None, use_errno=True)
        libc.prctl(1, signal.SIGTERM, 0, 0, 0)  # PR_SET_PDEATHSIG
    except (OSError, AttributeError):
        pass


# read at library load by OpenBLAS / OpenMP / MKL: the zygote imports with one-thread pools
_POOL_ENV = ("OPENBLAS_NUM_THREADS", "GOTO_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS")


def _native_threads() -> list[str]:
    """Names of this process's OS threads (/proc/self/task/*/comm), the main thread first."""
    out = []
    try:
        tids = sorted(os.listdir("/proc/self/task"), key=lambda t: (int(t) != os.getpid(), int(t)))
    except OSError:
        return ["?"]
    for t in tids:
        try:
            with open(f"/proc/self/task/{t}/comm") as f:
                out.append(f"{t}:{f.read().strip()}")
        except OSError:
            pass
    return out


def _env_threads(env: dict, *keys: str) -> int:
    for k in keys:
        try:
            n = int(env.get(k) or 0)
        except ValueError:
            n = 0
        if n > 0:
            return n
    return len(os.sched_getaffinity(0))


def _size_thread_pools(env: dict) -> None:
    """The OpenMP / OpenBLAS runtimes read their thread counts when the zygote loaded them (pinned to
    one, see _POOL_ENV), so a forked container would keep that instead of what a fresh process pinned
    to its NUMA-local CPUs gets. Apply the container's own settings, as a fresh process would read them."""
    torch = sys.modules.get("torch")
    if torch is not None:
        torch.set_num_threads(max(1, _env_threads(env, "OMP_NUM_THREADS")))
    if "numpy" in sys.modules:
        try:
            from threadpoolctl import threadpool_limits
            threadpool_limits(_env_threads(env, "OPENBLAS_NUM_THREADS", "GOTO_NUM_THREADS", "OMP_NUM_THREADS"),
                              user_api="blas")
        except Exception:  # noqa: BLE001 - no threadpoolctl in this image: BLAS stays single-threaded
            pass


def _join_netns(path: str) -> None:
    """Enter the pod's network namespace (kubelet --pod-netns) before any of the container's code
    runs; a container that cannot be isolated must not run at all (the exception exits the child)."""
    import ctypes
    fd = os.open(path, os.O_RDONLY | os.O_CLOEXEC)
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        if libc.setns(fd, 0x40000000) != 0:  # CLONE_NEWNET
            err = ctypes.get_errno()
            raise OSError(err, f"setns({path}): {os.strerror(err)}")
    finally:
        os.close(fd)


# env read when HIP / ROCr / comgr initialise: a warm child serves a request only if these match
_HIP_ENV_PREFIXES = ("ROCR_", "HIP_", "HSA_", "GPU_", "CUDA_", "AMD_", "PYTORCH_")
_HIP_ENV_IGNORE = {"AMD_COMGR_CACHE_DIR", "AMD_COMGR_CACHE"}


def _hip_env(env: dict) -> dict:
    return {k: v for k, v in env.items() if k.startswith(_HIP_ENV_PREFIXES) and k not in _HIP_ENV_IGNORE}


def _warm_env(dev: int) -> dict:
    """The env a warm child initialises the GPU under: the zygote's (the kubelet's pass-through
    HSA_* / ROCm settings) plus the device plugin's 1-GPU view of device `dev`."""
    env = {k: v for k, v in os.environ.items() if k not in _POOL_ENV}
    for k in [k for k in env if k.startswith(_HIP_ENV_PREFIXES)]:
        if k.endswith("VISIBLE_DEVICES") or k == "GPU_DEVICE_ORDINAL":
            del env[k]
    env.update({"ROCR_VISIBLE_DEVICES": str(dev), "HIP_VISIBLE_DEVICES": "0",
                # no comgr cache while warming: the cache dir is per tenant and this child has none yet
                "AMD_COMGR_CACHE": "0"})
    return env


def _warm_child(dev: int, ctl: socket.socket, closefds: list[int]) -> None:
    """Runs in a forked warm child: bring the GPU up, report, wait for a container request on `ctl`,
    then become that container (_child). Never returns."""
    try:
        gc.enable()
        for fd in closefds:
            try:
                os.close(fd)
            except OSError:
                pass
        signal.set_wakeup_fd(-1)
        try:
            import ctypes
            ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGKILL, 0, 0, 0)  # dies with the zygote until claimed
        except (OSError, AttributeError):
            pass
        env = _warm_env(dev)
        os.environ.clear()
        os.environ.update(env)
        t0 = time.perf_counter()
        import torch
        torch.cuda.init()
        x = torch.zeros(1 << 20, device="cuda")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        steps = {"device_ms": round((t1 - t0) * 1e3, 1)}
        try:  # the notebook server's first GEMM shape: its code object is resident before the pod exists
            from kubeflow_rm_amd import ops
            a = torch.ones(1024, 1024, device="cuda", dtype=torch.bfloat16)
            ops.gemm_nt(a, a)
            torch.cuda.synchronize()
            steps["kernels_ms"] = round((time.perf_counter() - t1) * 1e3, 1)
        except Exception as e:  # noqa: BLE001 - the container loads them itself then
            steps["kernels_error"] = f"{type(e).__name__}: {e}"
        del x
        ctl.sendall((json.dumps({"ready": True, "device": dev, "env": _hip_env(env), **steps}) + "\n").encode())
        buf = b""
        while not buf.endswith(b"\n"):
            chunk = ctl.recv(65536)
            if not chunk:
                os._exit(0)  # the zygote went away or retired this child
            buf += chunk
        req = json.loads(buf)
    except BaseException as e:  # noqa: BLE001 - a child that cannot warm up says so and leaves
        try:
            ctl.sendall((json.dumps({"ready": False, "error": f"{type(e).__name__}: {e}"}) + "\n").encode())
        except OSError:
            pass
        os._exit(1)
    try:
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(1, 0, 0, 0, 0)  # claimed: lives like any container
    except (OSError, AttributeError):
        pass
    _child(req, [ctl.fileno()], warm=True)


def _child(req: dict, closefds: list[int], warm: bool = False) -> None:
    """Runs in the forked process (or a claimed warm child): become the container, run its module,
    never return."""
    code = 1
    try:
        gc.enable()
        for fd in closefds:
            try:
                os.close(fd)
            except OSError:
                pass
        signal.set_wakeup_fd(-1)
        if req.get("netns"):
            _join_netns(req["netns"])
        os.setsid()
        for s in (signal.SIGTERM, signal.SIGCHLD, signal.SIGHUP, signal.SIGPIPE, signal.SIGQUIT):
            signal.signal(s, signal.SIG_DFL)
        signal.signal(signal.SIGINT, signal.default_int_handler)
        signal.pthread_sigmask(signal.SIG_SETMASK, [])
        cpus = [c for c in req.get("cpus") or [] if isinstance(c, int)]
        if cpus:
            # a warm child already runs the GPU runtime's threads: every thread gets the mask
            for tid in (os.listdir("/proc/self/task") if warm else ["0"]):
                try:
                    os.sched_setaffinity(int(tid), cpus)
                except OSError:
                    pass
        fd = os.open(req["log"], os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        nul = os.open(os.devnull, os.O_RDONLY)
        os.dup2(nul, 0)
        os.dup2(fd, 1)
        os.dup2(fd, 2)
        os.close(fd)
        os.close(nul)
        os.chdir(req["cwd"])
        env = dict(kv.split("=", 1) for kv in req.get("env") or [] if "=" in kv)
        os.environ.clear()
        os.environ.update(env)
        pp = [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p]
        sys.path[:0] = [p for p in pp if p not in sys.path]
        _size_thread_pools(env)
        argv = list(req["argv"])
        if len(argv) < 2 or argv[0] != "-m":
            raise ValueError(f"zygote runs 'python -m module' containers only, got {argv!r}")
        sys.argv = [argv[1]] + argv[2:]
        print(f"[zygote] pid {os.getpid()} runs {argv[1]} (preloaded: {sorted(_PRELOADED)})", flush=True)
        # executed afresh as __main__ (its own imports stay cached); a preloaded copy in sys.modules
        # would only make runpy warn
        sys.modules.pop(argv[1], None)
        runpy.run_module(argv[1], run_name="__main__", alter_sys=True)
        code = 0
    except SystemExit as e:
        code = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
        if e.code is not None and not isinstance(e.code, int):
            print(e.code, file=sys.stderr)
    except BaseException:  # noqa: BLE001 - the container's crash, reported like python would
        traceback.print_exc()
        code = 1
    finally:
        try:
            sys.stdout.flush()
            sys.stderr.flush()
        except Exception:  # noqa: BLE001
            pass
        os._exit(code & 0xFF)


_PRELOADED: set[str] = set()


def serve(sock_path: str, preload: list[str], warm_devices: list[int] | None = None,
          warm_modules: list[str] | None = None) -> int:
    t0 = time.perf_counter()
    # pre-fork server idiom (Python docs, gc.freeze): no collections while the preload allocates (no
    # freed holes in shared pages), then every preloaded object moves to the permanent generation, so a
    # container's collections never write the gc headers of the shared copies (copy-on-write faults on
    # the cold-start path); each child re-enables gc first thing
    gc.disable()
    for mod in preload:
        importlib.import_module(mod)
        _PRELOADED.add(mod)
    gc.freeze()
    import_s = time.perf_counter() - t0
    if _gpu_driver_open():
        print(f"[zygote] refusing to serve: preloading {preload} opened the GPU driver", flush=True)
        return 3
    threads = _native_threads()
    if len(threads) > 1:
        print(f"[zygote] refusing to serve: preloading {preload} left {len(threads)} threads {threads}; "
              "a fork would copy only the main one", flush=True)
        return 4
    _set_pdeathsig()
    try:
        os.unlink(sock_path)
    except FileNotFoundError:
        pass
    lsock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    try:
        os.unlink(sock_path + ".tmp")
    except FileNotFoundError:
        pass
    lsock.bind(sock_path + ".tmp")
    # only the kubelet's user may ask for a process (a request names the env, cwd and log file)
    os.chmod(sock_path + ".tmp", 0o600)
    lsock.listen(64)
    os.rename(sock_path + ".tmp", sock_path)  # the socket appears only once the zygote accepts
    print(f"[zygote] pid {os.getpid()} ready on {sock_path}: preloaded {preload} in {import_s:.2f} s, "
          f"threads {len(_native_threads())}", flush=True)

    rd, wr = os.pipe()
    os.set_blocking(rd, False)
    os.set_blocking(wr, False)
    signal.set_wakeup_fd(wr)
    signal.signal(signal.SIGCHLD, lambda *_: None)
    stop = []
    signal.signal(signal.SIGTERM, lambda *_: stop.append(1))
    sel = selectors.DefaultSelector()
    sel.register(lsock, selectors.EVENT_READ, "listen")
    sel.register(rd, selectors.EVENT_READ, "sigchld")
    children: dict[int, socket.socket] = {}
    warm_devices = list(warm_devices or [])
    warm_modules = set(warm_modules or [])
    # device -> {"pid", "sock", "ready": bool, "env": {...}}; at most one per device
    warm: dict[int, dict] = {}
    warm_failures: dict[int, int] = {}
    warm_due: dict[int, float] = {}  # device -> when to fork its next warm child (after a claim)

    def start_warm(dev: int) -> None:
        if dev in warm or warm_failures.get(dev, 0) >= 3 or stop:
            return
        if len(_native_threads()) > 1:
            return
        parent, child = socket.socketpair()
        sys.stdout.flush()
        sys.stderr.flush()
        pid = os.fork()
        if pid == 0:
            parent.close()
            _warm_child(dev, child, [lsock.fileno(), rd, wr] + [c.fileno() for c in children.values()] +
                        [w["sock"].fileno() for w in warm.values()])
        child.close()
        warm[dev] = {"pid": pid, "sock": parent, "ready": False, "started": time.perf_counter()}
        sel.register(parent, selectors.EVENT_READ, ("warm", dev))

    def warm_message(dev: int) -> None:
        w = warm.get(dev)
        if w is None:
            return
        try:
            line = w["sock"].recv(65536)
        except OSError:
            line = b""
        msg = {}
        try:
            msg = json.loads(line) if line else {}
        except ValueError:
            pass
        if msg.get("ready"):
            w["ready"] = True
            w["env"] = msg.get("env") or {}
            warm_failures[dev] = 0
            print(f"[zygote] warm child {w['pid']} for device {dev} ready in "
                  f"{(time.perf_counter() - w['started']) * 1e3:.0f} ms {msg}", flush=True)
            return
        print(f"[zygote] warm child {w['pid']} for device {dev} failed: {msg.get('error') or 'exited'}", flush=True)
        retire(dev)
        warm_failures[dev] = warm_failures.get(dev, 0) + 1

    def retire(dev: int) -> None:
        w = warm.pop(dev, None)
        if w is None:
            return
        try:
            sel.unregister(w["sock"])
        except (KeyError, ValueError):
            pass
        w["sock"].close()  # an unclaimed child exits on EOF

    def claim(dev: int, req: dict, conn: socket.socket) -> bool:
        """Hand `req` to the warm child of `dev` if it is ready (waiting up to 0.3 s for one that is
        still warming) and its GPU env matches the request's."""
        w = warm.get(dev)
        if w is None:
            return False
        deadline = time.perf_counter() + 0.3
        while not w["ready"] and time.perf_counter() < deadline:
            r, _, _ = select.select([w["sock"]], [], [], max(0.0, deadline - time.perf_counter()))
            if r:
                warm_message(dev)
                w = warm.get(dev)
                if w is None:
                    return False
        if not w["ready"]:
            return False
        env = dict(kv.split("=", 1) for kv in req.get("env") or [] if "=" in kv)
        if _hip_env(env) != w["env"]:
            print(f"[zygote] warm child for device {dev} not used: GPU env differs "
                  f"({sorted(set(_hip_env(env).items()) ^ set(w['env'].items()))[:6]})", flush=True)
            return False
        try:
            w["sock"].sendall((json.dumps(req) + "\n").encode())
        except OSError:
            retire(dev)
            return False
        pid = w["pid"]
        try:
            sel.unregister(w["sock"])
        except (KeyError, ValueError):
            pass
        w["sock"].close()
        del warm[dev]
        children[pid] = conn
        conn.settimeout(None)
        try:
            conn.sendall((json.dumps({"pid": pid, "warm": True}) + "\n").encode())
        except OSError:
            pass
        # the next one warms up once this container's own GPU start is past (no KFD contention on its
        # cold-start path)
        warm_due[dev] = time.perf_counter() + 0.3
        return True

    def reap():
        while True:
            try:
                pid, st = os.waitpid(-1, os.WNOHANG)
            except ChildProcessError:
                return
            if pid == 0:
                return
            conn = children.pop(pid, None)
            if conn is None:
                continue
            sig = os.WTERMSIG(st) if os.WIFSIGNALED(st) else 0
            code = os.WEXITSTATUS(st) if os.WIFEXITED(st) else 128 + sig
            try:
                conn.sendall((json.dumps({"exit": code, "signal": sig}) + "\n").encode())
            except OSError:
                pass
            conn.close()

    def handle(conn: socket.socket):
        conn.settimeout(5)
        buf = b""
        try:
            while not buf.endswith(b"\n"):
                chunk = conn.recv(65536)
                if not chunk:
                    break
                buf += chunk
            req = json.loads(buf)
            argv = req.get("argv") if isinstance(req, dict) else None
            if not (isinstance(argv, list) and len(argv) >= 2 and argv[0] == "-m" and
                    all(isinstance(x, str) for x in argv) and isinstance(req.get("cwd"), str) and
                    isinstance(req.get("log"), str) and isinstance(req.get("env", []), list)):
                raise ValueError("want {argv: ['-m', module, ...], cwd, log, env, cpus}")
        except (OSError, ValueError) as e:
            try:
                conn.sendall((json.dumps({"error": f"bad request: {e}"}) + "\n").encode())
            except OSError:
                pass
            conn.close()
            return
        dev = req.get("warm_device")
        if (isinstance(dev, int) and dev in warm and len(argv) >= 2 and argv[1] in warm_modules
                and claim(dev, req, conn)):
            return
        sys.stdout.flush()
        sys.stderr.flush()
        threads = _native_threads()
        if len(threads) > 1:  # started since the preload check: never fork around it
            print(f"[zygote] not forking: {len(threads)} threads {threads}", flush=True)
            try:
                conn.sendall((json.dumps({"error": f"zygote is multi-threaded ({len(threads)})"}) + "\n").encode())
            except OSError:
                pass
            conn.close()
            stop.append(1)
            return
        pid = os.fork()
        if pid == 0:
            _child(req, [lsock.fileno(), rd, wr] + [c.fileno() for c in children.values()] + [conn.fileno()] +
                   [w["sock"].fileno() for w in warm.values()])
        children[pid] = conn
        conn.settimeout(None)
        try:
            conn.sendall((json.dumps({"pid": pid}) + "\n").encode())
        except OSError:
            pass

    for d in warm_devices:
        start_warm(d)
    while not stop:
        now = time.perf_counter()
        timeout = min([1.0] + [max(0.0, t - now) for t in warm_due.values()])
        for key, _ in sel.select(timeout=timeout):
            if isinstance(key.data, tuple):  # a warm child's report (or its exit)
                warm_message(key.data[1])
                continue
            if key.data == "listen":
                try:
                    conn, _ = lsock.accept()
                except OSError:
                    continue
                handle(conn)
            else:
                try:
                    while os.read(rd, 4096):
                        pass
                except (BlockingIOError, OSError):
                    pass
        reap()
        now = time.perf_counter()
        for d in warm_devices:  # a claimed / retired / failed warm child is replaced (at most 3 failures in a row)
            if d not in warm and warm_due.get(d, 0.0) <= now:
                warm_due.pop(d, None)
                start_warm(d)
    for d in list(warm):
        retire(d)
    try:
        os.unlink(sock_path)
    except OSError:
        pass
    return 0


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="pre-imported interpreter for process pods")
    p.add_argument("--socket", required=True)
    p.add_argument("--preload", default="", help="comma-separated modules to import before serving")
    p.add_argument("--warm-devices", default="", help="comma-separated node GPU ids to keep a warm child for")
    p.add_argument("--warm-modules", default="kubeflow_rm_amd.images.notebook_server",
                   help="comma-separated container modules a warm child may become")
    a = p.parse_args(argv)
    for k in _POOL_ENV:  # the containers get their own env; these only shape the preload
        os.environ[k] = "1"
    return serve(a.socket, [m for m in a.preload.split(",") if m],
                 [int(d) for d in a.warm_devices.split(",") if d.strip()], [m for m in a.warm_modules.split(",") if m])


if __name__ == "__main__":
    sys.exit(main())
