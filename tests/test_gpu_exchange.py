"""The label exchange's device path on one GPU (distributed.LabelExchange, the RCCL branch): the
two ranks' exchange objects live in one process and a loopback transport stands in for RCCL.

RCCL cannot run two ranks on one GPU, so the driver's N > 1 runs are the first to move labels
over xGMI. What this file checks on the GPU is everything around the transport that the RCCL
branch adds: the sender narrows a tile's label planes into its per-tile wire buffers on its send
stream behind the tile's completion event; the writer receives into wire buffers on its receive
stream and widens them there; wait() makes the caller's stream wait for those copies. The loopback
transport moves the bytes stream-ordered the way RCCL's stream does: a send records an event on
the stream it is posted from, the matching receive waits for it on the receive stream.
"""
import pytest
import torch

from land_trendr_amd import distributed as ltd
from land_trendr_amd.runner import label_wire_types
from land_trendr_amd.settings import compile_params

pytestmark = pytest.mark.gpu

RULES = [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
         {'name': 'fd', 'val': 2, 'change_type': 'FD', 'duration': ['<', 5]}]


class _Work:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):  # as ProcessGroupNCCL's Work: the current stream waits, the host does not
        torch.cuda.current_stream().wait_event(self.ev)


class _Loopback:
    """batch_isend_irecv between exchange objects of one process (sends must be posted first)."""
    isend, irecv = 'send', 'recv'

    def __init__(self):
        self.sends = []
        self.bytes = 0

    @staticmethod
    def P2POp(op, tensor, peer):
        return (op, tensor, peer)

    @staticmethod
    def get_backend():
        return 'nccl'

    def batch_isend_irecv(self, ops):
        works = []
        for op, t, _ in ops:
            ev = torch.cuda.Event()
            if op == 'send':
                ev.record()
                self.sends.append((t, ev))
            else:
                src, sev = self.sends.pop(0)
                assert src.dtype == t.dtype and src.shape == t.shape
                torch.cuda.current_stream().wait_event(sev)
                t.copy_(src)
                self.bytes += t.numel() * t.element_size()
                ev.record()
            works.append(_Work(ev))
        return works


def _spec(R):
    return {'class_val': (R, torch.int32), 'onset_year': (R, torch.int32),
            'duration': (R, torch.int32), 'magnitude': (R, torch.float64)}


@pytest.mark.parametrize('overlap', [False, True])
def test_narrow_label_transfer_streams(overlap):
    """Rank 1's tile goes to writer rank 0 in three steps, with new labels each step; the
    writer's rasters equal the sender's planes bit for bit after every step (joined), or after
    the last one (pipelined: the sender's next kernels wait only for that tile's last send)."""
    dev = torch.device('cuda', 0)
    W, R = 1 << 20, 2
    params, _ = compile_params(10, RULES)
    wire = label_wire_types(params, tuple(_spec(R)))
    assert set(wire) == {'class_val', 'onset_year', 'duration'}
    loop = _Loopback()
    ex = [ltd.LabelExchange(ltd.Mosaic([W, W], W, 2, r, 'round_robin'), _spec(R), dev, loop, 0,
                            wire) for r in (0, 1)]
    writer, sender = ex
    assert writer.is_writer and not sender.is_writer and sender.can_overlap
    g = torch.Generator(device=dev).manual_seed(5)
    main = torch.cuda.current_stream(dev)
    want = {}
    for step in range(3):
        for k, t in enumerate(sender.m.mine):
            if overlap:  # runner._wait_sends: this tile's previous send before its kernels
                sender.wait_round(k)
            s = sender.slab(t)
            # "the kernels": new labels written on the main stream, a done event after them
            s['class_val'].copy_(torch.randint(-99, 3, (R, W), device=dev, generator=g))
            s['onset_year'].copy_(torch.randint(1984, 2015, (R, W), device=dev, generator=g))
            s['duration'].copy_(torch.randint(-99, 31, (R, W), device=dev, generator=g))
            s['magnitude'].copy_(torch.randn((R, W), device=dev, generator=g, dtype=torch.float64))
            want[t.t] = {f: x.clone() for f, x in s.items()}
            done = torch.cuda.Event()
            done.record(main)
            sender.post(k, after=done)
            # the writer computes tile 0 itself; its own slabs are not received
            writer.post(k)
        if not overlap:
            sender.wait()
            writer.wait()
            _check(writer, want, step)
    sender.wait()
    writer.wait()
    _check(writer, want, 'last')
    # the wire carried 2 + 2 + 2 + 8 bytes per pixel and rule
    assert loop.bytes == 3 * R * W * 14


def _check(writer, want, step):
    torch.cuda.synchronize()
    for t, planes in want.items():
        for f, x in planes.items():
            y = writer.full[f][t]
            assert y.dtype == x.dtype
            same = (y.view(torch.int64) == x.view(torch.int64)) if f == 'magnitude' else y == x
            assert bool(same.all()), (step, t, f)
