"""roctx range helper: no-op when disabled or without a GPU, balanced push/pop when enabled."""


def test_trace_range_noop_and_enabled(monkeypatch):
    from ddp_amd.utils import trace
    calls = []

    class FakeNvtx:
        def range_push(self, n):
            calls.append(("push", n))

        def range_pop(self):
            calls.append(("pop",))

        def mark(self, n):
            calls.append(("mark", n))

    trace.enable(False)
    with trace.trace_range("forward"):
        pass
    assert calls == []
    monkeypatch.setattr(trace, "_nvtx", lambda: FakeNvtx())
    trace.enable(True)
    try:
        with trace.trace_range("backward"):
            trace.mark("bucket0")
    finally:
        trace.enable(False)
    assert calls == [("push", "backward"), ("mark", "bucket0"), ("pop",)]
