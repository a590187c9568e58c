"""Fallback ladder for multi-rank benchmark runs: a failed attempt is retried with a simpler
gradient-synchronisation plan in FRESH processes, so one bug in an advanced path cannot leave a
multi-GPU run without a number.

The reference's DDP run (/root/reference/part3/main.py:159-186) has one execution plan. Here the
planned multi-GPU step (pipelined segments, start-up collective probe, cut planner, sharded
update) has more moving parts than the plain captured DDP step, and a failure inside any of them
(a rank that exits, a watchdog that fires on a hung collective, replicas that diverge) would end
the whole run. ``bench.py`` therefore runs the ranks as attempts of a ladder:

    attempt 0  "planned"     the arguments as given
    attempt 1  "inline-ddp"  one captured graph per step, bucket all-reduces inline
                             (--segmented 0 --update allreduce, no start-up probe / cut planner)
    attempt 2  "eager"       the same without hipGraph capture (--no-graph)

Every attempt is a new set of rank processes (never an ``exec``: the supervising process makes
no GPU call at all). Two supervisors:

* ``run_self`` — ``bench.py --gpus N`` without an outer launcher: this process spawns the N
  ranks of each attempt itself (utils/launch.py conventions: own session per rank, parent-death
  signal, a failing rank stops its peers after a grace period, overall timeout per attempt).
* ``run_under_launcher`` — one rank of an outer launcher (the driver's ``torchrun
  --nproc-per-node N bench.py``): each of the N launcher ranks supervises ONE child, its own
  rank of the attempt. The supervisors form a Gloo group on the launcher's rendezvous (CPU
  only) and coordinate through its store: rank 0 picks a fresh rendezvous port per attempt (the
  children host their own store there), a failing child raises the attempt's failure counter
  and every other supervisor stops its child after the grace period, and all agree on the
  outcome before the next attempt starts.

Rank 0's JSON line is printed once, by the supervisor, with ``"attempts"``: one record per
attempt run (name, ok, and for failures the reason and the failing rank's stderr tail).
"""
import collections
import json
import os
import subprocess
import sys
import threading
import time

from .launch import _SignalGuard, _child_setup, _kill_all, check_no_gpu_init, free_port, rank_env

# set in every attempt's ranks (they run, not supervise): the attempt index (fault injection)
ATTEMPT_ENV = CHILD_ENV = "DDP_AMD_LADDER_ATTEMPT"
# exit codes of a rank that ran to the end but whose result must not be reported
RC_REPLICAS = 5    # replicas not bit-identical after the timed steps
RC_WATCHDOG = 3    # utils/misc.py Watchdog


def default_attempts(strategy="ddp"):
    """The ladder for a bench strategy (list of {name, args, env})."""
    simple_env = {"DDP_AMD_COMM_PROBE": "0", "DDP_AMD_CUT_PLAN": "0"}
    if strategy != "ddp":  # 2A / 2B have no pipelined plan: captured, then eager
        return [{"name": "planned", "args": [], "env": {}},
                {"name": "eager", "args": ["--no-graph"], "env": simple_env}]
    return [{"name": "planned", "args": [], "env": {}},
            {"name": "inline-ddp", "args": ["--segmented", "0", "--update", "allreduce"],
             "env": simple_env},
            {"name": "eager", "args": ["--segmented", "0", "--update", "allreduce", "--no-graph"],
             "env": simple_env}]


def _reason_for(rc):
    if rc == RC_REPLICAS:
        return f"exit {rc}: replicas not bit-identical"
    if rc == RC_WATCHDOG:
        return f"exit {rc}: watchdog (no progress / RCCL async error)"
    if rc is not None and rc < 0:
        return f"killed by signal {-rc}"
    return f"exit {rc}"


class _Pump(threading.Thread):
    """Reads a child's pipe line by line: forwards each line to ``sink`` (except JSON lines
    when ``hold_json``) and keeps the last ``keep`` lines and every JSON line."""

    def __init__(self, pipe, sink, hold_json=False, keep=40):
        super().__init__(daemon=True)
        self.pipe, self.sink, self.hold_json = pipe, sink, hold_json
        self.tail = collections.deque(maxlen=keep)
        self.json = []

    def run(self):
        for raw in iter(self.pipe.readline, b""):
            line = raw.decode(errors="replace").rstrip("\n")
            if self.hold_json and line.startswith("{"):
                try:
                    json.loads(line)
                    self.json.append(line)
                    continue
                except ValueError:
                    pass
            self.tail.append(line)
            try:
                self.sink.write(line + "\n")
                self.sink.flush()
            except (OSError, ValueError):
                pass
        self.pipe.close()

    def text(self, chars=2000):
        return "\n".join(self.tail)[-chars:]


def _spawn(cmd, env, capture_json):
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         start_new_session=True, preexec_fn=_child_setup)
    out = _Pump(p.stdout, sys.stderr, hold_json=capture_json)
    err = _Pump(p.stderr, sys.stderr)
    out.start()
    err.start()
    return p, out, err


def _child_env(base, attempt_index, extra):
    env = dict(base)
    env.update(extra)
    env[ATTEMPT_ENV] = str(attempt_index)
    # a hung collective must end the attempt well inside the supervisor's time limit
    env.setdefault("DDP_AMD_WATCHDOG_S", "120")
    return env


def _finish(record, json_lines, log):
    """Rank 0's JSON line with the attempt records added (None if there is none)."""
    if not json_lines:
        return None
    d = json.loads(json_lines[-1])
    d["attempts"] = record
    if len(record) > 1:
        log(f"result from attempt {len(record) - 1} ({record[-1]['name']}) after "
            f"{len(record) - 1} failed attempt(s)")
    return json.dumps(d)


def _log_default(m):
    print(f"[ladder] {m}", file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------- self launch
def run_self(script, argv, nprocs, attempts, timeout_s=480.0, grace_s=15.0, addr="127.0.0.1",
             log=None, poll_s=0.05):
    """Run ``script argv`` as ``nprocs`` ranks per attempt until one attempt succeeds. Prints the
    successful attempt's JSON line (with ``attempts``) on stdout; returns the exit code (0, or
    the last attempt's failure code)."""
    log = log or _log_default
    check_no_gpu_init()
    record, rc_last = [], 1
    for i, at in enumerate(attempts):
        port = free_port(addr)
        cmd = [sys.executable, os.path.abspath(script)] + list(argv) + list(at["args"])
        log(f"attempt {i} ({at['name']}): {nprocs} ranks")
        procs, pumps = [], []
        guard = _SignalGuard(procs, log)
        reason, bad_rank, rc_fail = None, None, 0
        try:
            guard.__enter__()
            for r in range(nprocs):
                env = _child_env(rank_env(r, nprocs, port, addr), i, at["env"])
                p, out, err = _spawn(cmd, env, capture_json=(r == 0))
                procs.append(p)
                pumps.append((out, err))
            t0, failed_at = time.monotonic(), None
            while True:
                codes = [p.poll() for p in procs]
                if all(c is not None for c in codes):
                    bad = [(r, c) for r, c in enumerate(codes) if c != 0]
                    if bad and reason is None:
                        bad_rank, rc_fail = bad[0]
                        reason = _reason_for(rc_fail)
                    break
                bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
                if bad and failed_at is None:
                    failed_at = time.monotonic()
                    bad_rank, rc_fail = bad[0]
                    reason = _reason_for(rc_fail)
                    log(f"rank {bad_rank}: {reason}; stopping the others in {grace_s:g}s")
                if failed_at is not None and time.monotonic() - failed_at > grace_s:
                    _kill_all(procs)
                    break
                if time.monotonic() - t0 > timeout_s:
                    reason, bad_rank, rc_fail = f"timeout after {timeout_s:g}s", None, 124
                    log(f"attempt {i}: {reason}: killing {nprocs} ranks")
                    _kill_all(procs)
                    break
                time.sleep(poll_s)
        except BaseException:
            _kill_all(procs)
            raise
        finally:
            guard.__exit__()
        for out, err in pumps:
            out.join(5.0)
            err.join(5.0)
        json_lines = pumps[0][0].json if pumps else []
        if reason is None and not json_lines:
            reason, bad_rank, rc_fail = "no JSON line from rank 0", 0, 1
        if reason is None:
            record.append({"name": at["name"], "ok": True})
            line = _finish(record, json_lines, log)
            print(line, flush=True)
            return 0
        tail_rank = bad_rank if bad_rank is not None else 0
        record.append({"name": at["name"], "ok": False, "reason": reason, "rank": bad_rank,
                       "stderr_tail": pumps[tail_rank][1].text() if pumps else ""})
        rc_last = rc_fail or 1
        log(f"attempt {i} ({at['name']}) failed: {reason}")
    print(json.dumps({"error": "every attempt failed", "attempts": record}), file=sys.stderr,
          flush=True)
    return rc_last


# ------------------------------------------------------------------------- under a launcher
def run_under_launcher(script, argv, attempts, timeout_s=480.0, grace_s=15.0, poll_s=0.2,
                       log=None):
    """This process is one rank of an outer launcher (torchrun): supervise this rank's child of
    every attempt (module docstring). Returns the exit code; launcher rank 0 prints the JSON."""
    import datetime
    import torch.distributed as dist
    log = log or _log_default
    check_no_gpu_init()
    # stdout carries exactly one line (the JSON): anything else (Gloo's connection messages,
    # the children's other output) goes to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=3600))
    rank, world = dist.get_rank(), dist.get_world_size()
    store = dist.PrefixStore("ddp_amd/ladder", dist.distributed_c10d._get_default_store())
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    record, rc_last = [], 1
    try:
        for i, at in enumerate(attempts):
            key = f"a{i}"
            if rank == 0:
                store.set(key + "/port", str(free_port(addr)))
            port = int(store.get(key + "/port"))
            env = _child_env(os.environ, i, at["env"])
            env["MASTER_PORT"] = str(port)
            env["MASTER_ADDR"] = addr
            env.pop("TORCHELASTIC_USE_AGENT_STORE", None)  # the children host their own store
            cmd = [sys.executable, os.path.abspath(script)] + list(argv) + list(at["args"])
            if rank == 0:
                log(f"attempt {i} ({at['name']}): {world} ranks")
            p, out, err = _spawn(cmd, env, capture_json=(rank == 0))
            t0, failed_at, reason = time.monotonic(), None, None
            guard = _SignalGuard([p], log)
            try:
                guard.__enter__()
                while True:
                    rc = p.poll()
                    if rc is not None:
                        if rc != 0:
                            reason = _reason_for(rc)
                        break
                    if failed_at is None and store.add(key + "/fail", 0) > 0:
                        failed_at = time.monotonic()
                    if failed_at is not None and time.monotonic() - failed_at > grace_s:
                        _kill_all([p])
                        reason = "stopped after a peer failed"
                        break
                    if time.monotonic() - t0 > timeout_s:
                        _kill_all([p])
                        reason = f"timeout after {timeout_s:g}s"
                        break
                    time.sleep(poll_s)
            except BaseException:
                _kill_all([p])
                raise
            finally:
                guard.__exit__()
            out.join(5.0)
            err.join(5.0)
            if reason is None and rank == 0 and not out.json:
                reason = "no JSON line from rank 0"
            if reason is not None:
                order = store.add(key + "/fail", 1)  # 1 = the first supervisor to see a failure
                store.set(f"{key}/reason/{rank}", json.dumps({"reason": reason, "order": order,
                                                             "tail": err.text()}))
            store.add(key + "/done", 1)
            deadline = time.monotonic() + timeout_s + 2 * grace_s + 60.0
            while store.add(key + "/done", 0) < world and time.monotonic() < deadline:
                time.sleep(poll_s)
            complete = store.add(key + "/done", 0) >= world
            if complete and store.add(key + "/fail", 0) == 0:
                record.append({"name": at["name"], "ok": True})
                if rank == 0:
                    print(_finish(record, out.json, log), file=json_out, flush=True)
                return 0
            # the rank whose failure was seen first names the attempt's failure (a rank stopped
            # because of a peer never does while another reason exists)
            rec = {"name": at["name"], "ok": False, "reason": "a supervisor did not finish",
                   "rank": None, "stderr_tail": ""}
            best = None
            for r in range(world):
                if not store.check([f"{key}/reason/{r}"]):
                    continue
                d = json.loads(store.get(f"{key}/reason/{r}"))
                k = (d["reason"] == "stopped after a peer failed", d["order"])
                if best is None or k < best:
                    best = k
                    rec.update(reason=d["reason"], rank=r, stderr_tail=d["tail"])
            record.append(rec)
            rc_last = 1
            if rank == 0:
                log(f"attempt {i} ({at['name']}) failed on rank {rec['rank']}: {rec['reason']}")
        if rank == 0:
            print(json.dumps({"error": "every attempt failed", "attempts": record}),
                  file=sys.stderr, flush=True)
        return rc_last
    finally:
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001 (best effort at exit)
            pass
