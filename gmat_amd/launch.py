"""One process per GPU without an external launcher (bench.py's contract).

``python bench.py --gpus N`` with no WORLD_SIZE in the environment starts N fresh child
processes of the same script, one per GPU, each with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set exactly as ``torch.distributed.run`` would set them, and waits for
them.  The parent never touches the GPU (it imports nothing from the HIP library): the children
are started before any HIP call in this process, so no GPU state is inherited or exec'd over.

The reference's own multi-process mode is the user-launched ``parallel=[N, k]`` split
(remma_epiAA.py:109-161): N independent invocations, one per part.  Here the parts are the
ranks of one job (dist.rank_rows) and their hits are merged on rank 0.

Failure behaviour: if any child exits non-zero, the others are terminated (their exact PIDs)
and the parent exits with the first failing child's code; a WORLD_SIZE that disagrees with
``--gpus`` is an error, never a silent single-rank run.
"""
import os
import signal
import socket
import subprocess
import sys
import time


class LaunchError(RuntimeError):
    pass


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def resolve(n_gpus, environ=None):
    """What this process is, given ``--gpus n_gpus``: "spawn" (no launcher: start n_gpus ranks),
    "single" (one process, no process group) or "rank" (a rank of an n_gpus-process job).
    Raises LaunchError when an existing WORLD_SIZE contradicts n_gpus."""
    env = os.environ if environ is None else environ
    if n_gpus < 1:
        raise LaunchError("--gpus %d: need at least one GPU" % n_gpus)
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if n_gpus > 1 else "single"
    ws = int(ws)
    if ws != n_gpus:
        raise LaunchError("--gpus %d but WORLD_SIZE=%d (set by the launcher): refusing to run a different number "
                          "of ranks than asked for" % (n_gpus, ws))
    return "rank" if ws > 1 else "single"


def rank_env(base, rank, world_size, port, addr="127.0.0.1"):
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world_size),
                "LOCAL_WORLD_SIZE": str(world_size), "GROUP_RANK": "0", "MASTER_ADDR": addr,
                "MASTER_PORT": str(port), "GMAT_LAUNCHER": "gmat_amd.launch"})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    return env


def spawn(argv, n_procs, environ=None, poll_s=0.2, timeout_s=None):
    """Run ``argv`` (a full command line, e.g. [sys.executable, script, ...]) as ranks 0..n_procs-1
    of one job and return 0, or the exit code of the first rank that failed (the others are
    terminated).  stdout / stderr are inherited: rank 0's JSON line reaches the caller's stdout."""
    base = dict(os.environ if environ is None else environ)
    port = int(base.get("MASTER_PORT") or free_port())
    procs = []
    try:
        for r in range(n_procs):
            procs.append(subprocess.Popen(argv, env=rank_env(base, r, n_procs, port)))
        t0 = time.time()
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print("gmat_amd.launch: rank %d exited with %d; stopping the other ranks" % (r, c), file=sys.stderr,
                      flush=True)
                return c if c > 0 else 128 - c
            if all(c == 0 for c in codes):
                return 0
            if timeout_s is not None and time.time() - t0 > timeout_s:
                print("gmat_amd.launch: ranks still running after %.0f s; stopping them" % timeout_s, file=sys.stderr,
                      flush=True)
                return 124
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()


def visible_devices(environ=None, timeout_s=180):
    """GPUs a rank of this job would see, counted in a CHILD process (hipGetDeviceCount initialises
    the runtime; the launcher itself must stay GPU-free because it starts the ranks).  0 when the
    library or the runtime reports none; None when the probe itself failed (timed out, crashed or
    printed nothing) -- then the count is unknown, which is not the CPU harness's 0."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from gmat_amd import _native as N\n"
            "lib = N.load(required=False)\n"
            "print(N.device_count() if lib is not None else 0)\n" % os.path.dirname(os.path.dirname(
                os.path.abspath(__file__))))
    env = dict(os.environ if environ is None else environ)
    env.pop("GMAT_NUM_GPUS", None)
    try:
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                             timeout=timeout_s)
        if out.returncode != 0 or not out.stdout.strip():
            return None
        return int(out.stdout.strip().splitlines()[-1])
    except (subprocess.TimeoutExpired, ValueError):
        return None


def check_devices(n_gpus, n_visible, allow_shared):
    """None when n_gpus ranks can each have a GPU of their own (or sharing is allowed, or the job
    runs on the CPU test harness with no GPU at all); else the error text.  n_visible None (the
    device probe failed) is refused unless sharing is allowed."""
    if allow_shared:
        return None
    if n_visible is None:
        return ("--gpus %d but the GPU count could not be probed (the child process failed): refusing to start "
                "ranks that may share a device (--allow-shared-gpu to start them anyway)" % n_gpus)
    if n_visible == 0 or n_visible >= n_gpus:
        return None
    return ("--gpus %d but only %d GPU(s) visible: one process per GPU, so the job would report GPUs it does not "
            "use (--allow-shared-gpu lets ranks share devices, for tests)" % (n_gpus, n_visible))


def main_or_spawn(n_gpus, script, argv, allow_shared=False):
    """bench.py's entry: returns None when this process should do the work itself (a single
    process, or a rank started by a launcher), else spawns the ranks and returns their exit
    code for the caller to exit with.  More ranks than visible GPUs is an error (exit status 2)
    unless allow_shared."""
    try:
        what = resolve(n_gpus)
    except LaunchError as exc:
        print("error: %s" % exc, file=sys.stderr, flush=True)
        return 2
    if what != "spawn":
        return None
    err = check_devices(n_gpus, visible_devices(), allow_shared)
    if err:
        print("error: %s" % err, file=sys.stderr, flush=True)
        return 2
    return spawn([sys.executable, script] + list(argv), n_gpus)


def _refuse(msg):
    print("error: %s" % msg, file=sys.stderr, flush=True)
    return 2


def spawn_from_env(environ=None, argv=None):
    """GMAT_NUM_GPUS=N (N > 1) with no WORLD_SIZE: start N ranks of this very command line (the script,
    ``-m module`` or ``-c code`` the interpreter was started with) and return their exit status; None
    when there is nothing to spawn.  Called when gmat_amd is first imported -- before the script makes
    any GPU call, so the parent stays GPU-free (it only waits).  The ranks then run the script as one
    job: the drop-in scans shard their work over the ranks, rank 0 writes the files (dist.job)."""
    env = os.environ if environ is None else environ
    raw = env.get("GMAT_NUM_GPUS", "").strip()
    if not raw or env.get("WORLD_SIZE") is not None:
        return None
    try:
        n = int(raw)
    except ValueError:
        return _refuse("GMAT_NUM_GPUS=%r is not an integer" % raw)
    if n < 1:
        return _refuse("GMAT_NUM_GPUS=%d: need at least one GPU" % n)
    if n == 1:
        return None
    cmd = list(sys.orig_argv[1:] if argv is None else argv)
    if not cmd or cmd[0] in ("-", "-i") or (not sys.argv or sys.argv[0] in ("", "-")):
        return _refuse("GMAT_NUM_GPUS=%d needs a script, -m module or -c code to start as %d ranks (not an "
                       "interactive or stdin session)" % (n, n))
    allow = env.get("GMAT_ALLOW_SHARED_GPU", "") not in ("", "0")
    err = check_devices(n, visible_devices(env), allow)
    if err:
        return _refuse(err)
    return spawn([sys.executable] + cmd, n, environ=env)


def main(argv=None):
    """``python -m gmat_amd.launch --gpus N [--allow-shared-gpu] script.py [args ...]`` (or ``-m module``):
    the script runs unchanged as N ranks of one job, one process per GPU (torchrun's environment)."""
    import argparse
    ap = argparse.ArgumentParser(prog="python -m gmat_amd.launch", description=main.__doc__)
    ap.add_argument("--gpus", type=int, required=True)
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="tests only: more ranks than visible GPUs (ranks share devices, exchanges over gloo)")
    ap.add_argument("-m", dest="module", default=None, help="run a module as the ranks' program")
    ap.add_argument("cmd", nargs=argparse.REMAINDER, help="script.py [args ...] (or the module's arguments)")
    a = ap.parse_args(argv)
    cmd = (["-m", a.module] if a.module else []) + list(a.cmd)
    if not cmd:
        return _refuse("nothing to run: give a script or -m module")
    if a.gpus < 1:
        return _refuse("--gpus %d: need at least one GPU" % a.gpus)
    base = dict(os.environ)
    base.pop("GMAT_NUM_GPUS", None)
    if a.allow_shared_gpu:
        base["GMAT_ALLOW_SHARED_GPU"] = "1"
    if a.gpus == 1:
        return subprocess.call([sys.executable] + cmd, env=base)
    err = check_devices(a.gpus, visible_devices(base), a.allow_shared_gpu)
    if err:
        return _refuse(err)
    return spawn([sys.executable] + cmd, a.gpus, environ=base)


if __name__ == "__main__":
    sys.exit(main())
