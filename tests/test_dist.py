"""The sharded multi-GPU path (config 5) on CPU: world_size 2 over gloo.

Each rank demodulates its contiguous shard of independent streams (here with
the oracle standing in for the GPU kernel: this test covers the sharding,
the symbol gather and rank-0 framing, not the kernel), gathers every rank's
symbols and rank 0 frames them into ToReceiver messages; the reassembled
stream must equal the single-process oracle result.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_streams, wps, k, q):
    try:
        _work(rank, world, port, n_streams, wps, k, q)
    except BaseException:
        import traceback
        q.put(("error", traceback.format_exc()))
        raise


def _work(rank, world, port, n_streams, wps, k, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from conftest import load_pkg
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    A = load_pkg()
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "audio_network_amd.dist", os.path.join(ROOT, "audio-network_amd", "dist.py"))
    D = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(D)
    freqs = A.FSK2_FREQS if k == 2 else A.FSK8_FREQS
    first, count = D.shard_range(n_streams, rank, world)
    pcm, _ = O.synth_fsk(freqs, 1024, count * wps, 0x2C5DA044, w0=first * wps)
    sym, _ = O.goertzel(pcm, freqs, 1024)
    full = D.gather_symbols(torch.from_numpy(sym), n_streams, world, unit=wps)
    if rank == 0:
        stream = D.frame_symbols(A, full.numpy(), k)
        back = D.unframe_symbols(A, stream, n_streams * wps, k)
        q.put((full.numpy().tobytes(), back.tobytes(), len(stream)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_streams,k", [(2, 6, 2), (2, 7, 8), (3, 5, 2)])
def test_sharded_demod_gather_and_framing(A, O, world, n_streams, k):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    wps = 40  # windows per stream
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_streams, wps, k, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    assert res[0] != "error", res[1]
    full, back, nbytes = res
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    freqs = A.FSK2_FREQS if k == 2 else A.FSK8_FREQS
    pcm, truth = O.synth_fsk(freqs, 1024, n_streams * wps, 0x2C5DA044)
    ref, _ = O.goertzel(pcm, freqs, 1024)
    got = np.frombuffer(full, np.uint8)
    assert (got == ref).all() and (got == truth).all()
    assert np.frombuffer(back, np.uint8).tolist() == ref.tolist()
    assert nbytes > 0


def test_shard_range_properties():
    sys.path.insert(0, ROOT)
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "dist_mod", os.path.join(ROOT, "audio-network_amd", "dist.py"))
    D = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(D)
    for total in (0, 1, 7, 1024, 1025):
        for world in (1, 2, 3, 8):
            spans = [D.shard_range(total, r, world) for r in range(world)]
            assert sum(c for _, c in spans) == total
            pos = 0
            for f, c in spans:
                assert f == pos
                pos += c
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _bucket_worker(rank, world, port, n_streams, wps, S, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import torch
        import torch.distributed as dist
        from conftest import load_pkg
        from oracle import oracle as O

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        A = load_pkg()
        import importlib.util
        spec = importlib.util.spec_from_file_location(
            "audio_network_amd.dist", os.path.join(ROOT, "audio-network_amd", "dist.py"))
        D = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(D)
        freqs, k = A.FSK2_FREQS, 2
        bits = A.bits_per_symbol(k)
        fstride = A.frame_symbols_size(wps, bits)
        first, count = D.shard_range(n_streams, rank, world)
        max_count = -(-n_streams // world)
        # S steps of this rank's streams, each stream's frames in its own
        # fstride slot, step-major: bench.py's bucket layout ([S][count])
        local = np.zeros(S * count * fstride, np.uint8)
        for s in range(S):
            pcm, _ = O.synth_fsk(freqs, 1024, count * wps, 0x5EED + s, w0=first * wps)
            sym, _ = O.goertzel(pcm, freqs, 1024)
            for j in range(count):
                fr = np.frombuffer(A.frame_symbols(sym[j * wps:(j + 1) * wps], bits), np.uint8)
                assert fr.size <= fstride
                off = (s * count + j) * fstride
                local[off:off + fr.size] = fr
        blocks = D.gather_blocks(torch.from_numpy(local), world, S * max_count * fstride)
        if rank == 0:
            q.put(blocks.numpy().tobytes())
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put(("error", traceback.format_exc()))
        raise


@pytest.mark.parametrize("world,n_streams", [(2, 6), (3, 7)])
def test_bucket_gather_blocks(A, O, world, n_streams):
    """configs[4]'s bucketed step on CPU (bench.py): every rank
    frames S steps of its (uneven) stream shard into one block, one
    gather_blocks all-gathers the padded blocks, and rank 0 decodes every
    rank's every step's every stream back to the oracle's symbols, as the
    bench's check of the last bucket does."""
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    sys.path.insert(0, ROOT)
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "dist_mod2", os.path.join(ROOT, "audio-network_amd", "dist.py"))
    D = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(D)
    wps, S = 24, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, n_streams, wps, S, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    assert not (isinstance(res, tuple) and res[0] == "error"), res[1]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    freqs, k = A.FSK2_FREQS, 2
    bits = A.bits_per_symbol(k)
    fstride = A.frame_symbols_size(wps, bits)
    max_count = -(-n_streams // world)
    blocks = np.frombuffer(res, np.uint8).reshape(world, S * max_count * fstride)
    for s in range(S):
        pcm, truth = O.synth_fsk(freqs, 1024, n_streams * wps, 0x5EED + s)
        tru = truth.reshape(n_streams, wps)
        for r in range(world):
            first, cnt = D.shard_range(n_streams, r, world)
            for j in range(cnt):
                off = (s * cnt + j) * fstride
                back = D.unframe_symbols(A, blocks[r][off:off + fstride].tobytes(), wps, k)
                assert (back == tru[first + j]).all(), (s, r, j)


def _settle_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        import torch
        import torch.distributed as dist
        import bench
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        clock = [0.0]

        class FakeCuda:
            @staticmethod
            def synchronize():
                pass

        class FakeTorch:
            cuda = FakeCuda

        class FakeTime:
            @staticmethod
            def perf_counter():
                return clock[0]
        bench.time = FakeTime
        # rank r's device ramps down from a transient for 3 r chunks of 4
        # steps (3.0, 2.85, ... ms per step), then runs at 2.0
        sched = [3.0 - 0.15 * c for c in range(3 * rank) for _ in range(4)] + [2.0] * 1000
        it = iter(sched)
        steps = [0]

        def fn():
            steps[0] += 1
            clock[0] += next(it) * 1e-3

        def agree(ok):
            t = torch.tensor([0.0 if ok else 1.0])
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item()) == 0.0
        n, times = bench.settle_warmup(FakeTorch, fn, chunk=4, agree=agree)
        q.put((rank, n, steps[0], times))
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put(("error", traceback.format_exc()))
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_settle_warmup_agreed_across_ranks(world):
    """bench.py's settle warmup at N > 1 (round 6): every step holds a
    collective, so the ranks must run the same number of warmup steps. Each
    rank's (fake) device settles after a different number of chunks; with
    the agreement (gloo all-reduce of each rank's verdict, as bench.py does
    on the device) every rank runs the slowest rank's count."""
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_settle_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
    assert all(r[0] != "error" for r in res), res
    counts = {r[1] for r in res} | {r[2] for r in res}
    assert len(counts) == 1, res                      # the same steps on every rank
    slowest = 3 * (world - 1) + 2                      # chunks until the last rank settles
    assert counts == {4 * slowest}, res
