"""Spawn world-N gloo process groups on 127.0.0.1 for the CPU tests of the
multi-rank host logic (tests only).

gloo's full-mesh connect occasionally loses a pair socket on a loaded host
("connectFullMesh failed ... Connection closed by peer"), before any test code
has run.  That is the transport's setup, not the logic under test, so a group
whose init fails is torn down and started again on a fresh port (at most
ATTEMPTS times); a failure after init is the test's and is never retried."""
import queue
import socket
import time

ATTEMPTS = 3


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(target, rank, world, port, args, q):
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    except Exception as e:  # noqa: BLE001 -- reported to the parent, which retries
        q.put(("init_failed", rank, repr(e)))
        return
    try:
        q.put(("ok", rank, target(rank, world, *args)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def run(target, world, args=(), timeout=120.0):
    """target(rank, world, *args) in `world` spawned ranks of one gloo group;
    returns the ranks' return values in rank order (picklable).  Retries only
    a group whose init_process_group failed."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    last = None
    for _ in range(ATTEMPTS):
        q = ctx.Queue()
        port = free_port()
        procs = [ctx.Process(target=_entry, args=(target, r, world, port, args, q)) for r in range(world)]
        for p in procs:
            p.start()
        got, failed = {}, None
        deadline = time.monotonic() + timeout
        try:
            while len(got) < world and failed is None:
                try:
                    kind, rank, val = q.get(timeout=1.0)
                except queue.Empty:
                    dead = [p for p in procs if p.exitcode not in (None, 0)]
                    if dead:
                        raise AssertionError(f"rank process exited with {dead[0].exitcode} before reporting")
                    if time.monotonic() > deadline:
                        raise AssertionError(f"ranks did not report within {timeout} s (got {sorted(got)})")
                    continue
                if kind == "init_failed":
                    failed = val
                else:
                    got[rank] = val
        finally:
            if failed is not None or len(got) < world:
                for p in procs:  # only the processes this call started
                    if p.is_alive():
                        p.terminate()
            for p in procs:
                p.join(timeout=60)
        if failed is None:
            for p in procs:
                assert p.exitcode == 0, p.exitcode
            return [got[r] for r in range(world)]
        last = failed
    raise AssertionError(f"gloo group init failed {ATTEMPTS} times: {last}")

