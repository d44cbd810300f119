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
process's parent) learns the exit status. The kubelet kills the process group (the child calls
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


def _child(req: dict, closefds: list[int]) -> None:
    """Runs in the forked process: become the container, run its module, never return."""
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
            try:
                os.sched_setaffinity(0, cpus)
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


def serve(sock_path: str, preload: list[str]) -> int:
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
            _child(req, [lsock.fileno(), rd, wr] + [c.fileno() for c in children.values()] + [conn.fileno()])
        children[pid] = conn
        conn.settimeout(None)
        try:
            conn.sendall((json.dumps({"pid": pid}) + "\n").encode())
        except OSError:
            pass

    while not stop:
        for key, _ in sel.select(timeout=1.0):
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
    try:
        os.unlink(sock_path)
    except OSError:
        pass
    return 0


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="pre-imported interpreter for process pods")
    p.add_argument("--socket", required=True)
    p.add_argument("--preload", default="", help="comma-separated modules to import before serving")
    a = p.parse_args(argv)
    for k in _POOL_ENV:  # the containers get their own env; these only shape the preload
        os.environ[k] = "1"
    return serve(a.socket, [m for m in a.preload.split(",") if m])


if __name__ == "__main__":
    sys.exit(main())
