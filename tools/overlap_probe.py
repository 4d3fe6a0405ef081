"""Does data movement make progress while the analyze kernel holds every CU? (VERDICT r04 item 4:
the label exchange at N > 1 is RCCL point-to-point, which runs as kernels needing CU slots.)

One GPU, bench.py's c2 launch (the JIT analyze kernel over one 49 Mpx scene), timed alone, then
with a concurrent transfer on another stream started at the same moment:
  * d2d_blit: a device-to-device copy of the c2 N = 8 writer ingress per step (7 x 49 Mpx x 20 B
    = 6.9 GB), torch copy_ (HIP's blit kernel: needs CU slots, as RCCL's kernels do);
  * d2h_sdma: a device-to-host copy into pinned memory (2 GB; the DMA engines, no CU slots).
For each: the analyze step's time with the transfer beside it, the transfer's own time alone and
when it completes relative to the step (an event on its stream). Prints one JSON object.
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from land_trendr_amd.distributed import Mosaic  # noqa: E402
from land_trendr_amd.engine import get_engine  # noqa: E402
from land_trendr_amd.index_eqn import IndexProgram  # noqa: E402
from land_trendr_amd.runner import MosaicRunner  # noqa: E402
from land_trendr_amd.settings import compile_params  # noqa: E402
from land_trendr_amd.synth import mosaic_inputs  # noqa: E402


def main():
    c = bench.CONFIGS['c2']
    P = c['pixels']
    dev = torch.device('cuda', 0)
    eng = get_engine(0)
    m = Mosaic([P], P, 1, 0, 'by_scene')
    items = mosaic_inputs(m, c['years'], 1, 1, 0.0, c['seed'], dev, bench.TARGET)
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))
    fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']
    r = MosaicRunner(eng, m, params, items, fields, fn)
    r.prepare_jit(wait=True)
    r.step()
    torch.cuda.synchronize()

    def step_time(n=3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            r.step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    alone = step_time()
    side = torch.cuda.Stream(dev)
    ing = 7 * P * 20
    src = torch.empty(ing, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    dsrc = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
    hdst = torch.empty(2 << 30, dtype=torch.uint8, pin_memory=True)
    res = {'analyze_step_alone_ms': round(alone, 3), 'pixels': P}
    for name, (a, b) in {'d2d_blit': (dst, src), 'd2h_sdma': (hdst, dsrc)}.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            e0.record()
            a.copy_(b, non_blocking=True)
            e1.record()
        torch.cuda.synchronize()
        t_alone = e0.elapsed_time(e1)
        # both at once: the transfer queued first on its stream, the step right after
        s0 = torch.cuda.Event(enable_timing=True)
        x0, x1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        m0, m1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s0.record()
        side.wait_event(s0)
        with torch.cuda.stream(side):
            x0.record()
            a.copy_(b, non_blocking=True)
            x1.record()
        m0.record()
        r.step()
        m1.record()
        torch.cuda.synchronize()
        res[name] = {'bytes': a.numel(), 'alone_ms': round(t_alone, 3),
                     'alone_gbs': round(a.numel() / t_alone / 1e6, 1),
                     'with_step': {'step_ms': round(m0.elapsed_time(m1), 3),
                                   'transfer_done_after_ms': round(s0.elapsed_time(x1), 3),
                                   'transfer_ms': round(x0.elapsed_time(x1), 3)}}
    # the exchange's real timing: a transfer queued when tile 0 is done, while tile 1's analyze
    # kernel holds the CUs (16.8 Mpx tiles, one call, per-tile completion events as runner.py
    # uses them at N > 1); per tile round the writer's ingress at N = 8 is 7 x 16.8 Mpx x 20 B
    m3 = Mosaic([P], 1 << 24, 1, 0, 'by_scene')
    items3 = mosaic_inputs(m3, c['years'], 1, 1, 0.0, c['seed'], dev, bench.TARGET)
    r3 = MosaicRunner(eng, m3, params, items3, fields, fn, None, exchange_fields=())
    r3.gathering = True
    r3.step()
    torch.cuda.synchronize()
    n3 = 7 * (1 << 24) * 20
    a, b = dst[:n3], src[:n3]
    for name, prio in (('blit_after_tile0', 0), ('blit_after_tile0_high_priority', -1)):
        st = torch.cuda.Stream(dev, priority=prio)
        marks = []

        def timed_events(n):  # the runner's per-tile completion events, with timing
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
            for e in evs:
                e.record()
            marks.extend(evs)
            return evs
        r3._done_events = timed_events
        s0, x1, t_end = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        torch.cuda.synchronize()
        s0.record()
        r3.step()  # queues all tiles; marks = their completion events
        st.wait_event(marks[0])
        with torch.cuda.stream(st):
            a.copy_(b, non_blocking=True)
            x1.record()
        t_end.record()
        torch.cuda.synchronize()
        del r3._done_events  # back to the class method
        res[name] = {'bytes': n3, 'step_ms': round(s0.elapsed_time(t_end), 3),
                     'tiles_done_ms': [round(s0.elapsed_time(e), 3) for e in marks],
                     'transfer_done_after_ms': round(s0.elapsed_time(x1), 3),
                     'note': 'tiles 16.8 Mpx x 3; the copy waits for tile 0'}
    # the same with the analyze / resolve launches on a CU-masked stream that leaves `free` CUs
    # (the mask's last bits) to the transfer (hipExtStreamCreateWithCUMask): does a reserved
    # slice let the blit (RCCL's P2P kernels likewise) progress beside analyze, and what does the
    # analyze step lose?
    import ctypes
    hip = ctypes.CDLL('libamdhip64.so')
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    for free in (8, 16):
        words = (n_cu + 31) // 32
        mask = (ctypes.c_uint32 * words)()
        for cu in range(n_cu - free):
            mask[cu // 32] |= 1 << (cu % 32)
        hs = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(hs), ctypes.c_uint32(words), mask)
        if rc != 0:
            res['cumask_error'] = rc
            break
        ms = torch.cuda.ExternalStream(hs.value, device=dev)
        with torch.cuda.stream(ms):
            r3.step()
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(3):
                r3.step()
            t1.record()
            torch.cuda.synchronize()
            masked_alone = t0.elapsed_time(t1) / 3
            marks = []

            def timed_events2(n):
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
                for e in evs:
                    e.record()
                marks.extend(evs)
                return evs
            r3._done_events = timed_events2
            s0, x1, t_end = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            torch.cuda.synchronize()
            s0.record()
            r3.step()
            side.wait_event(marks[0])
            with torch.cuda.stream(side):
                a.copy_(b, non_blocking=True)
                x1.record()
            t_end.record()
            torch.cuda.synchronize()
            del r3._done_events
        res['cumask_free%d' % free] = {
            'cus': n_cu, 'free_cus': free, 'step_alone_masked_ms': round(masked_alone, 3),
            'step_ms': round(s0.elapsed_time(t_end), 3),
            'tiles_done_ms': [round(s0.elapsed_time(e), 3) for e in marks],
            'transfer_done_after_ms': round(s0.elapsed_time(x1), 3)}
        torch.cuda.synchronize()
        hip.hipStreamDestroy(hs)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
