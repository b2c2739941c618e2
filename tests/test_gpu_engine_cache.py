"""The engine pool behind the blst-named entry points (csrc/pool.hpp) bounds
device memory by the peak number of CONCURRENT calls, not by the number of
threads that ever called -- a Go caller's pool of OS threads (blst.go:2105-2167)
used to pin one engine per thread until the thread exited."""
import ctypes
import threading

import pytest

pytestmark = pytest.mark.gpu

N = 1 << 12


@pytest.fixture()
def m():
    import msm_blst_amd as m
    m.release_engine_cache()
    assert m.engine_cache_stats()[0] == 0
    yield m
    m.set_engine_cache_limit(8 << 30)
    m.release_engine_cache()


def _call(m, pts, sc, out):
    pp = (ctypes.c_void_p * 2)(ctypes.cast(pts, ctypes.c_void_p), None)
    sp = (ctypes.c_void_p * 2)(ctypes.cast(sc, ctypes.c_void_p), None)
    r = (ctypes.c_uint8 * 144)()
    m.lib().blst_p1s_mult_pippenger(r, pp, N, sp, 255, None)
    out.append(m.compress(1, bytes(r)).hex())


def _golden(golden):
    return [c for c in golden("msm_g1.json")["cases"]
            if c["n"] == N and c["seed"] == 1 and c["case"] == "rand" and c["nbits"] == 255][0]["compressed"]


def test_many_threads_one_at_a_time_share_one_engine(m, golden, points):
    """24 long-lived threads each call once, never two at a time: one engine."""
    pts, sc = points(1, N), m.gen_scalars(N, 1)
    out, turn, stop = [], threading.Lock(), threading.Event()
    go = [threading.Event() for _ in range(24)]

    def worker(k):
        go[k].wait()
        with turn:
            _call(m, pts, sc, out)
        stop.wait()  # the thread stays alive, like a pooled OS thread

    th = [threading.Thread(target=worker, args=(k,)) for k in range(24)]
    for t in th:
        t.start()
    for k in range(24):
        go[k].set()
        while len(out) <= k:
            threading.Event().wait(0.001)
    live, idle, idle_bytes = m.engine_cache_stats()
    stop.set()
    for t in th:
        t.join()
    assert out == [_golden(golden)] * 24
    assert (live, idle) == (1, 1) and idle_bytes > 0


def test_concurrent_calls_are_bounded_and_released(m, golden, points):
    """8 concurrent callers: at most 8 engines; all equal the golden; release
    frees every idle engine; with a zero cache limit nothing stays cached."""
    pts, sc = points(1, N), m.gen_scalars(N, 1)
    out, bar = [], threading.Barrier(8)

    def worker():
        bar.wait()
        for _ in range(3):
            _call(m, pts, sc, out)

    th = [threading.Thread(target=worker) for _ in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert out == [_golden(golden)] * 24
    live, idle, _ = m.engine_cache_stats()
    assert 1 <= live <= 8 and idle == live
    m.release_engine_cache()
    assert m.engine_cache_stats() == (0, 0, 0)
    m.set_engine_cache_limit(0)
    out.clear()
    _call(m, pts, sc, out)
    assert out == [_golden(golden)]
    assert m.engine_cache_stats() == (0, 0, 0)


def test_lowered_limit_trims_idle_engines(m, golden, points):
    """msm_set_engine_cache_limit trims engines that are already idle (the
    limit is read atomically by every returning call, csrc/pool.hpp)."""
    pts, sc = points(1, N), m.gen_scalars(N, 1)
    out = []
    _call(m, pts, sc, out)
    assert m.engine_cache_stats()[:2] == (1, 1)
    m.set_engine_cache_limit(0)
    assert m.engine_cache_stats() == (0, 0, 0)
    assert out == [_golden(golden)]


def test_small_calls_hold_no_large_pinned_ring(m, points):
    """A 2^12-point call uploads < 1 MiB per buffer: no pinned ring is
    allocated, so the cached engine holds only its device buffers (the ring was
    a fixed 64 MiB per engine, counted nowhere)."""
    pts, sc = points(1, N), m.gen_scalars(N, 1)
    _call(m, pts, sc, [])
    _, idle, idle_bytes = m.engine_cache_stats()
    assert idle == 1 and 0 < idle_bytes < (64 << 20)


def test_failed_call_drops_its_engine(m, golden, points):
    """A call that throws after leasing its engine (nbits > 256 is rejected on
    the device path) must not return the engine to the pool: it is drained and
    destroyed during unwinding.  The next call gets a fresh engine and the
    golden result."""
    pts, sc = points(1, N), m.gen_scalars(N, 1)
    L = m.lib()
    prev = L.msm_set_abort_on_error(0)
    try:
        wide = (ctypes.c_uint8 * (N * 40))()
        pp = (ctypes.c_void_p * 2)(ctypes.cast(pts, ctypes.c_void_p), None)
        sp = (ctypes.c_void_p * 2)(ctypes.cast(wide, ctypes.c_void_p), None)
        r = (ctypes.c_uint8 * 144)()
        L.blst_p1s_mult_pippenger(r, pp, N, sp, 300, None)
        assert L.msm_error_pending()
        L.msm_last_error()
        assert m.engine_cache_stats() == (0, 0, 0)
    finally:
        L.msm_set_abort_on_error(prev)
    out = []
    _call(m, pts, sc, out)
    assert out == [_golden(golden)]
