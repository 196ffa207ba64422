"""StepThrottle (endossl/throttle.py): a trainer's next step waits for the step `depth` before it
(host run-ahead bound).  CUDA events are faked: this checks the bookkeeping only."""
import importlib

import torch

from endossl import throttle


class _Ev:
    log = []
    count = 0

    def __init__(self):
        self.id = _Ev.count
        _Ev.count += 1
        _Ev.log.append(("new", self.id))

    def record(self, stream=None):
        _Ev.log.append(("record", self.id))

    def synchronize(self):
        _Ev.log.append(("sync", self.id))


def _fake_cuda(monkeypatch):
    _Ev.log, _Ev.count = [], 0
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "Event", _Ev)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a: None)


def _run(th, steps):
    for _ in range(steps):
        th.wait()
        th.record()
    return [x for x in _Ev.log if x[0] == "sync"]


def test_depth_one_waits_for_the_previous_step(monkeypatch):
    _fake_cuda(monkeypatch)
    assert _run(throttle.StepThrottle(1), 3) == [("sync", 0), ("sync", 1)]


def test_depth_two_keeps_one_step_queued(monkeypatch):
    _fake_cuda(monkeypatch)
    assert _run(throttle.StepThrottle(2), 4) == [("sync", 0), ("sync", 1)]


def test_depth_zero_is_unbounded(monkeypatch):
    _fake_cuda(monkeypatch)
    assert _run(throttle.StepThrottle(0), 4) == [] and _Ev.log == []


def test_env_overrides_every_default(monkeypatch):
    monkeypatch.setenv("ENDOSSL_MAX_INFLIGHT_STEPS", "3")
    mod = importlib.reload(throttle)
    try:
        assert mod.StepThrottle(1).depth == 3 and mod.StepThrottle(2).depth == 3
    finally:
        monkeypatch.delenv("ENDOSSL_MAX_INFLIGHT_STEPS")
        importlib.reload(throttle)
    assert throttle.StepThrottle(2).depth == 2
