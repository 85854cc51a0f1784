"""Per-iteration gradient sinks for the model's activated tensors.

A training iteration renders several views of one model; every view's backward kernels (the
rasterizer's preprocess backward, the relit features' backward, the regularisers') produce a
full-size gradient of the same activated tensors (positions, scales, rotations, opacity,
materials), and autograd would sum them with one elementwise add per contribution.  With a
sink the producing kernels add into one buffer per tensor themselves (their ``accumulate``
bits, include/gsr.h GSR_ACC_*): the first producer stores, the later ones add.  The
producers run on the views' HIP streams, so every claim waits for the previous producer's
event and records its own: the read-modify-writes are ordered in launch order.  The
activations' backward (train._Activations) then reads the buffers.

A tensor is sink-tagged by ``GradSink`` (attribute ``_gsr_sink``); a producer that finds
the tag on its input writes there and returns no gradient to autograd for that input."""
from __future__ import annotations

from typing import Dict, Iterable, Optional, Tuple

import torch

# accumulate bits of the C ABI (include/gsr.h GSR_ACC_*), by the sink key they add into
ACC_BITS = {"xyz": 1, "scaling": 2, "rotation": 4, "opacity": 8, "albedo": 16, "roughness": 32, "metalness": 64}


class GradSink:
    def __init__(self, tensors: Dict[str, torch.Tensor]):
        dev = next(iter(tensors.values())).device
        self.device = dev
        self.buf: Dict[str, torch.Tensor] = {k: torch.empty(t.shape, dtype=torch.float32, device=dev)
                                             for k, t in tensors.items()}
        self.written = set()
        self.event: Optional[torch.cuda.Event] = None
        self.streams = set()
        for k, t in tensors.items():
            t._gsr_sink = (self, k)

    def claim(self, keys: Iterable[str]) -> Tuple[Dict[str, torch.Tensor], int]:
        """Before a producer's launch on the current stream: its output buffers and the
        accumulate bits (keys an earlier producer already wrote)."""
        s = torch.cuda.current_stream(self.device)
        if self.event is not None:
            s.wait_event(self.event)
        if s.cuda_stream not in self.streams:
            self.streams.add(s.cuda_stream)
            for b in self.buf.values():
                b.record_stream(s)
        keys = list(keys)
        acc = 0
        for k in keys:
            if k in self.written:
                acc |= ACC_BITS[k]
        return {k: self.buf[k] for k in keys}, acc

    def done(self, keys: Iterable[str]) -> None:
        """After the producer's launch: its keys are written; the next claim waits for it."""
        self.written.update(keys)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.event = ev

    def take(self, key: str) -> Optional[torch.Tensor]:
        """The summed gradient of ``key`` for a consumer on the current stream (None if no
        producer wrote it)."""
        if key not in self.written:
            return None
        if self.event is not None:
            torch.cuda.current_stream(self.device).wait_event(self.event)
        return self.buf[key]


def sink_of(t) -> Tuple[Optional[GradSink], Optional[str]]:
    tag = getattr(t, "_gsr_sink", None) if t is not None else None
    return tag if tag is not None else (None, None)


def outputs(inputs, need):
    """Producer helper.  inputs: the producer's input tensors with a gradient output each;
    need: whether each wants a gradient.  Claims the sink keys of the tagged ones (all tagged
    inputs of one producer share one sink) and returns (buffers: the sink buffer or None per
    input, returned: whether the gradient still goes to autograd, sink, keys claimed,
    accumulate bits)."""
    sink, keys = None, []
    for t, nd in zip(inputs, need):
        s, k = sink_of(t)
        if nd and s is not None:
            sink = s
            keys.append(k)
    bufs, acc = sink.claim(keys) if sink is not None else ({}, 0)
    outs, ret = [], []
    for t, nd in zip(inputs, need):
        s, k = sink_of(t)
        tagged = nd and s is not None
        outs.append(bufs[k] if tagged else None)
        ret.append(bool(nd) and not tagged)
    return outs, ret, sink, keys, acc
