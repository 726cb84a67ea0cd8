"""Host-memory frees are deferred while a persistent rollout is being paced
(population/runner.py): hipHostFree waits for the whole device, and during
pacing the device waits for the host, so a free there (a garbage-collected
runner's buffers finalised inside another runner's env step) would stall the
rollout until its timeout.  CPU test with a stand-in library."""

import pytest


class _FakeLib:
    def __init__(self):
        self.freed = []
        self.bufs = []

    def agx_host_alloc(self, nbytes):
        import ctypes

        b = ctypes.create_string_buffer(nbytes)
        self.bufs.append(b)
        return ctypes.addressof(b)

    def agx_host_free(self, p):
        self.freed.append(p)
        return 0


@pytest.fixture
def runner_mod(monkeypatch):
    from agilerl_amd.population import runner

    fake = _FakeLib()
    monkeypatch.setattr(runner._lib, "load", lambda *a, **k: fake)
    monkeypatch.setattr(runner, "_PACING", 0)
    monkeypatch.setattr(runner, "_DEFERRED_FREES", [])
    monkeypatch.setattr(runner, "_HOST_POOL", {})
    fake.syncs = 0

    def sync():
        fake.syncs += 1

    monkeypatch.setattr(runner, "_device_sync", sync)
    return runner, fake


def test_free_outside_pacing_is_immediate(runner_mod):
    runner, fake = runner_mod
    runner._host_free(11)
    assert fake.freed == [11]


def test_free_during_pacing_waits_for_the_outermost_end(runner_mod):
    runner, fake = runner_mod
    runner._pacing_begin()
    runner._host_free(1)
    runner._pacing_begin()  # nested (a second runner paced from inside the first's window)
    runner._host_free(2)
    runner._pacing_end()
    assert fake.freed == []
    runner._pacing_end()
    assert sorted(fake.freed) == [1, 2] and runner._DEFERRED_FREES == []
    runner._host_free(3)
    assert fake.freed[-1] == 3


def test_finalizer_of_a_collected_owner_is_deferred(runner_mod):
    import gc
    import weakref

    runner, fake = runner_mod

    class Owner:
        pass

    o = Owner()
    weakref.finalize(o, runner._host_free, 42)
    runner._pacing_begin()
    del o
    gc.collect()
    assert fake.freed == []
    runner._pacing_end()
    assert fake.freed == [42]


def test_pooled_buffer_reused_only_after_the_device_drains(runner_mod):
    """A retired runner's staging goes back to the size pool; the next owner
    takes it only after a device sync (queued work of the old owner may still
    touch it), zeroed, and never while a rollout is being paced."""
    import gc

    runner, fake = runner_mod

    class Owner:
        pass

    a = Owner()
    t = runner._coherent(a, 64)
    addr = t.data_ptr()
    t.fill_(7)
    del t, a
    gc.collect()
    assert runner._HOST_POOL[64] == [addr] and fake.syncs == 0
    runner._pacing_begin()
    b = Owner()
    tb = runner._coherent(b, 64)  # inside a pacing window: a fresh buffer, no sync
    assert tb.data_ptr() != addr and fake.syncs == 0 and runner._HOST_POOL[64] == [addr]
    runner._pacing_end()
    c = Owner()
    tc = runner._coherent(c, 64)
    assert tc.data_ptr() == addr and fake.syncs == 1 and int(tc.sum()) == 0
