"""C2 signal propagation (parallel/signals.py) and rank liveness (parallel/health.py) on gloo,
world 3, host shards.

* A watcher on rank 0 -- a plain local store read, as splinter_get_signal_count / `watch --group`
  do -- sees a pulse of a key owned by rank 2 without any caller running a collective.
* One rank dies mid-batch: the survivors, blocked in a collective, exit non-zero
  (EXIT_PEER_LOST) within the liveness timeout instead of hanging.
"""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_sharded_gloo import _keys


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sig_worker(rank, world, port, base, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from libsplinter_amd import Store, unlink
        from libsplinter_amd.parallel.sharded import HostShard, ShardedKV
        from libsplinter_amd.parallel.signals import SignalSync
        name = f"{base}_s{rank}"
        st = Store.create(name, slots=512, max_val=64, embeddings=False)
        kv = ShardedKV(HostShard(st))
        # a key owned by the LAST rank
        cands = [f"sig{i}" for i in range(200)]
        own = kv.owned_mask(_keys(cands))  # mask w.r.t. THIS rank; find the last rank's key via hashes
        from libsplinter_amd.parallel.sharded import shard_of
        owner = shard_of(kv.local.hash_keys(_keys(cands)), world).tolist()
        key = next(c for c, o in zip(cands, owner) if o == world - 1)
        del own
        if rank == world - 1:
            st.set(key, b"x")
            st.watch(key, 5)  # the watcher's group lives in the owner's slot
        sync = SignalSync(kv.local, period_ms=10)
        dist.barrier()
        c0 = st.signal_count(5)
        dist.barrier()
        if rank == world - 1:
            for _ in range(3):
                st.bump(key)  # local pulses on the owner shard only
        # rank 0's local view catches up without any collective of its own
        deadline = time.time() + 20
        while st.signal_count(5) < c0 + 3 and time.time() < deadline:
            time.sleep(0.01)
        got = st.signal_count(5) - c0
        time.sleep(0.1)
        dist.barrier()
        sync.stop()
        assert sync.error is None, repr(sync.error)
        assert got == 3, (rank, got)
        assert st.signal_count(5) - c0 == 3  # no double counting after more rounds
        q.put((rank, "ok"))
        st.close()
        unlink(name)
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_signal_sync_world3(uniq):
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sig_worker, args=(r, world, port, uniq, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(60)
    assert all(v == "ok" for v in res.values()), res


def _dead_worker(rank, world, port, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=600))
    from libsplinter_amd.parallel.health import Liveness, guarded
    Liveness(period_s=0.2, timeout_s=2.0)
    dist.barrier()
    if rank == 2:
        if mode == "exit":
            os._exit(0)  # dies mid-batch, without a word: peers see their sockets reset
        import signal
        os.kill(os.getpid(), signal.SIGSTOP)  # hangs: sockets stay open, heartbeats stop
    t = torch.ones(1 << 10)
    guarded(dist.all_reduce, t)  # cannot complete: rank 2 is gone (gloo timeout is 600 s)
    os._exit(0)


def _run_dead(mode):
    from libsplinter_amd.parallel.health import EXIT_PEER_LOST
    world = 3
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_dead_worker, args=(r, world, port, mode)) for r in range(world)]
    t0 = time.time()
    for p in ps:
        p.start()
    for p in ps[:2]:
        p.join(120)
    took = time.time() - t0
    codes = [p.exitcode for p in ps[:2]]
    for p in ps:
        if p.is_alive():
            p.kill()
            p.join(10)
    assert codes == [EXIT_PEER_LOST, EXIT_PEER_LOST], codes
    assert took < 90
    return ps[2].exitcode


def test_dead_rank_survivors_exit_nonzero():
    """Rank 2 exits mid-batch: the collective error becomes EXIT_PEER_LOST (guarded)."""
    assert _run_dead("exit") == 0


def test_hung_rank_survivors_exit_nonzero():
    """Rank 2 hangs (SIGSTOP, connections open): the collective would block for the gloo
    timeout; the liveness monitor sees the stale heartbeat and ends the survivors."""
    _run_dead("hang")


def test_guarded_reraises_local_errors():
    """A local failure inside the step (HIP OOM, launch failure, shape bug) is not a lost peer:
    guarded() lets it propagate instead of exiting with EXIT_PEER_LOST."""
    from libsplinter_amd.parallel.health import guarded

    def oom():
        raise RuntimeError("HIP out of memory. Tried to allocate 2.00 GiB")

    def shape():
        raise ValueError("shape mismatch")

    with pytest.raises(RuntimeError, match="out of memory"):
        guarded(oom)
    with pytest.raises(ValueError):
        guarded(shape)
    assert guarded(lambda x: x + 1, 41) == 42
