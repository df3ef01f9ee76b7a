"""Multi-process launcher for CPU (gloo) distributed tests."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _port_race(err):
    # free_port() releases the port before rank 0 binds it: under pytest-xdist another test's
    # launcher can take it in between (EADDRINUSE) -- a harness race, retried once
    return "EADDRINUSE" in str(err)


def run_workers(module, world, args=(), timeout=240, env_extra=None):
    """Run `python -m tests.workers.<module> args...` on `world` ranks; returns outputs.
    Raises AssertionError with the logs if any rank fails."""
    try:
        return _run_workers(module, world, args, timeout, env_extra)
    except AssertionError as e:
        if not _port_race(e):
            raise
        return _run_workers(module, world, args, timeout, env_extra)


def _run_workers(module, world, args=(), timeout=240, env_extra=None):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update(RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SMP_FORCE_CPU="1", SMP_LOG_LEVEL="warning",
                   PYTHONPATH=ROOT + os.pathsep + env.get("PYTHONPATH", ""), OMP_NUM_THREADS="1",
                   SMP_CONNECT_TIMEOUT="60")
        if env_extra:
            env.update({k: str(v) for k, v in env_extra.items()})
            if "LOCAL_WORLD_SIZE" in env_extra:  # emulate several nodes of LOCAL_WORLD_SIZE ranks
                env["LOCAL_RANK"] = str(r % int(env_extra["LOCAL_WORLD_SIZE"]))
        procs.append(subprocess.Popen([sys.executable, "-m", f"tests.workers.{module}", *map(str, args)], cwd=ROOT,
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs, failed = [], False
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            o = "TIMEOUT\n" + (p.communicate()[0] or "")
            failed = True
        outs.append(o)
        if p.returncode != 0:
            failed = True
    if failed:
        msg = "\n".join(f"===== rank {i} (rc={p.returncode}) =====\n{o[-6000:]}" for i, (p, o) in enumerate(zip(procs, outs)))
        raise AssertionError(msg)
    return outs


def run_script(path, world, args=(), timeout=240, env_extra=None):
    """Run a repository script on `world` ranks (same env contract as run_workers)."""
    try:
        return _run_script(path, world, args, timeout, env_extra)
    except AssertionError as e:
        if not _port_race(e):
            raise
        return _run_script(path, world, args, timeout, env_extra)


def _run_script(path, world, args=(), timeout=240, env_extra=None):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update(RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SMP_FORCE_CPU="1", SMP_LOG_LEVEL="warning",
                   PYTHONPATH=ROOT + os.pathsep + env.get("PYTHONPATH", ""), OMP_NUM_THREADS="1",
                   SMP_CONNECT_TIMEOUT="60")
        env.update({k: str(v) for k, v in (env_extra or {}).items()})
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, path), *map(str, args)], cwd=ROOT, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs, failed = [], False
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            o = "TIMEOUT\n" + (p.communicate()[0] or "")
            failed = True
        outs.append(o)
        failed = failed or p.returncode != 0
    if failed:
        raise AssertionError("\n".join(f"===== rank {i} (rc={p.returncode}) =====\n{o[-5000:]}"
                                       for i, (p, o) in enumerate(zip(procs, outs))))
    return outs
