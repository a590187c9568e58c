"""One-process-per-GPU self-launcher (no outer torchrun needed).

The reference starts one process per node by hand, each with ``--num-nodes/--rank``
(/root/reference/README.md:8-19, /root/reference/part3/main.py:160-167). On one MI355X node the
equivalent is one process per GPU; ``bench.py --gpus N`` and ``tools/comm_bench.py --gpus N``
use this module when no launcher set ``WORLD_SIZE``:

* the parent makes NO GPU call (it may count devices: ``torch.cuda.device_count()`` does not
  initialise HIP on this image) and never ``exec``s — it spawns N children with
  ``subprocess`` and waits for them;
* each child gets ``RANK = LOCAL_RANK = r``, ``WORLD_SIZE = LOCAL_WORLD_SIZE = N``,
  ``MASTER_ADDR`` (127.0.0.1) and one free ``MASTER_PORT`` shared by all, plus
  ``DDP_AMD_LAUNCHER=self`` (recorded in the bench JSON);
* only rank 0's stdout reaches the parent's stdout (the one JSON line); the other ranks'
  stdout goes to stderr;
* every child runs in its own session: on a child failure (after a grace period for its
  peers to notice) or on the overall timeout the parent kills every child's process group and
  returns non-zero (the failing rank's code, or 124 on timeout);
* the ranks never outlive the launcher: SIGTERM / SIGHUP / SIGINT to the parent kill every
  rank's process group before the parent exits with 128 + signal, and each child also carries
  a parent-death signal (``prctl(PR_SET_PDEATHSIG, SIGKILL)``), which covers a parent killed
  with SIGKILL — the ranks would otherwise keep their GPUs and RCCL communicators.
"""
import ctypes
import os
import signal
import socket
import subprocess
import sys
import time


def free_port(addr="127.0.0.1"):
    """A TCP port that was free a moment ago on ``addr`` (the rendezvous store binds it)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def under_launcher():
    """True when an outer launcher (torchrun, this module, a job script) already set the env."""
    return "WORLD_SIZE" in os.environ


def check_no_gpu_init():
    """The parent must not have touched the GPU before spawning (a HIP context in the parent
    would pin memory on GPU 0 and, on this pool, forbids exec-style hand-offs)."""
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        raise RuntimeError("launcher parent initialised the GPU before spawning its ranks")


def visible_devices():
    import torch
    return torch.cuda.device_count()


def rank_env(rank, world, port, addr="127.0.0.1", base=None):
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "ROLE_RANK": str(rank),
                "MASTER_ADDR": addr, "MASTER_PORT": str(port), "DDP_AMD_LAUNCHER": "self"})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes)
    return env


_PR_SET_PDEATHSIG = 1


def _child_setup():
    """preexec_fn of every rank (runs in the forked child before exec): SIGKILL when the
    launcher dies, whatever kills it."""
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        libc.prctl(_PR_SET_PDEATHSIG, signal.SIGKILL, 0, 0, 0)
    except (OSError, AttributeError):
        pass


class _SignalGuard:
    """Within the ``with`` block, SIGTERM / SIGHUP / SIGINT kill the ranks, then exit the parent
    with 128 + signal (only installable from the main thread; a no-op elsewhere)."""

    SIGNALS = (signal.SIGTERM, signal.SIGHUP, signal.SIGINT)

    def __init__(self, procs, log):
        self.procs, self.log, self.old = procs, log, {}

    def _handler(self, signum, frame):
        self.log(f"launcher got signal {signum}: killing {len(self.procs)} ranks")
        _kill_all(self.procs)
        os._exit(128 + signum)

    def __enter__(self):
        import threading
        if threading.current_thread() is threading.main_thread():
            for s in self.SIGNALS:
                self.old[s] = signal.signal(s, self._handler)
        return self

    def __exit__(self, *exc):
        for s, h in self.old.items():
            signal.signal(s, h)
        return False


def spawn(cmd, nprocs, timeout_s=None, addr="127.0.0.1", port=None, grace_s=15.0, poll_s=0.05,
          log=None):
    """Run ``cmd`` (argv list) as ``nprocs`` ranks; return 0 when every rank exits 0, else the
    first failing rank's exit code (124 on timeout). ``log`` receives launcher messages
    (default stderr)."""
    log = log or (lambda m: print(f"[launch] {m}", file=sys.stderr, flush=True))
    check_no_gpu_init()
    port = port or free_port(addr)
    procs = []
    guard = _SignalGuard(procs, log)
    try:
        guard.__enter__()
        for r in range(nprocs):
            out = None if r == 0 else sys.stderr
            procs.append(subprocess.Popen(cmd, env=rank_env(r, nprocs, port, addr), stdout=out,
                                          start_new_session=True, preexec_fn=_child_setup))
        t0 = time.monotonic()
        failed_at, rc_fail = None, 0
        while True:
            codes = [p.poll() for p in procs]
            if all(c is not None for c in codes):
                bad = [(r, c) for r, c in enumerate(codes) if c != 0]
                if bad:
                    r, c = bad[0]
                    log(f"rank {r} exited with {c}")
                    return c if c > 0 else 128 - c
                return 0
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad and failed_at is None:
                failed_at, rc_fail = time.monotonic(), bad[0][1]
                log(f"rank {bad[0][0]} exited with {bad[0][1]}; stopping the others in {grace_s:g}s")
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                _kill_all(procs)
                return rc_fail if rc_fail > 0 else 128 - rc_fail
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                log(f"timeout after {timeout_s:g}s: killing {nprocs} ranks")
                _kill_all(procs)
                return 124
            time.sleep(poll_s)
    except BaseException:
        _kill_all(procs)
        raise
    finally:
        guard.__exit__()


def _kill_all(procs):
    for sig in (signal.SIGTERM, signal.SIGKILL):
        alive = [p for p in procs if p.poll() is None]
        if not alive:
            return
        for p in alive:
            try:
                os.killpg(p.pid, sig)  # the child's own session = its process group
            except ProcessLookupError:
                pass
        deadline = time.monotonic() + 5.0
        while time.monotonic() < deadline and any(p.poll() is None for p in alive):
            time.sleep(0.05)


def self_launch(script, argv, nprocs, timeout_s=None, require_devices=True):
    """Re-run ``script argv`` as ``nprocs`` ranks (see module docstring). Raises SystemExit with
    a clear message when fewer GPUs are visible than ranks requested."""
    if require_devices:
        n = visible_devices()
        if n < nprocs:
            raise SystemExit(f"--gpus {nprocs} but only {n} GPU(s) visible: refusing to run "
                             f"{nprocs} ranks on fewer devices")
    return spawn([sys.executable, os.path.abspath(script)] + list(argv), nprocs,
                 timeout_s=timeout_s)
