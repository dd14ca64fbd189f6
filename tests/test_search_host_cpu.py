"""CPU: host-side plumbing of the search pipeline (search.py) with the CUDA calls mocked: the
status / result staging records its event on the stream of the tensor's OWN device (an index on
cuda:1 while cuda:0 is current must not record on cuda:0's stream), and the pipeline enqueues
batch j + 1 before finishing batch j."""
import types

import torch

from denseretrievaltoolkits_amd import search


class _FakeTensor:
    def __init__(self, device):
        self.device = device
        self.shape = (4,)
        self.dtype = torch.int32
        self.is_cuda = True


def test_stage_host_records_on_the_tensors_device_stream(monkeypatch):
    calls = []

    class Stream:
        def __init__(self, dev):
            self.dev = dev

    class Event:
        def record(self, stream=None):
            calls.append(("record", stream.dev if stream is not None else "current"))

    class DeviceCtx:
        def __init__(self, dev):
            self.dev = dev

        def __enter__(self):
            calls.append(("enter", self.dev))

        def __exit__(self, *a):
            calls.append(("exit", self.dev))

    fake_cuda = types.SimpleNamespace(device=DeviceCtx, current_stream=lambda dev=None: Stream(dev), Event=Event)
    monkeypatch.setattr(search.torch, "cuda", fake_cuda)

    class Host:
        def copy_(self, t, non_blocking=False):
            calls.append(("copy", t.device, non_blocking))

    monkeypatch.setattr(search.torch, "empty", lambda *a, **k: Host())
    dev1 = torch.device("cuda", 1)
    hs, ev = search._stage_host(_FakeTensor(dev1), _FakeTensor(dev1))
    assert ("record", dev1) in calls
    assert calls[0] == ("enter", dev1) and calls[-1] == ("exit", dev1)
    assert [c for c in calls if c[0] == "copy"] == [("copy", dev1, True), ("copy", dev1, True)]


def test_pipeline_enqueues_next_before_finishing():
    log = []
    out = list(search._pipeline([10, 11, 12], lambda j, q: (log.append(("enq", j)), j)[1],
                                lambda j: (log.append(("fin", j)), j)[1]))
    assert out == [0, 1, 2]
    assert log == [("enq", 0), ("enq", 1), ("fin", 0), ("enq", 2), ("fin", 1), ("fin", 2)]
