"""Would two half-batch pipelines on two streams beat one full-batch step?  Times (a) the C3
8-view step graph, (b) two 4-view step graphs replayed one after the other, (c) the same two
replayed concurrently on two streams.  python tools/concurrency_probe.py [--tile-history 0|1]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kaolin_amd import _lib, distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tile-history', type=int, default=1)
    ap.add_argument('--steps', type=int, default=40)
    a = ap.parse_args()
    args = argparse.Namespace(config='c3', dtype='f32', knum=30, sigmainv=7000., boxlen=0.02,
                              iou=None, vertex_path='node', perturb=0.0)
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    _lib.load()
    _lib.set_tile_history(bool(a.tile_history))
    wa = bench.Workload(args, dev, 0, 4, 8)
    wb = bench.Workload(args, dev, 4, 4, 8)
    w8 = bench.Workload(args, dev, 0, 8, 8)
    ga = distributed.GraphedStep(wa.params, wa.forward_backward, params_to_reduce=[])
    gb = distributed.GraphedStep(wb.params, wb.forward_backward, params_to_reduce=[])
    g8 = distributed.GraphedStep(w8.params, w8.forward_backward, params_to_reduce=[])
    cur = torch.cuda.current_stream()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def seq():
        ga.replay()
        gb.replay()

    def conc():
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            gb.replay()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    def timed(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) * 1e3 / a.steps, 4)

    out = {'tile_history': a.tile_history}
    for rep in range(3):
        out[f'full8_{rep}'] = timed(g8.replay)
        out[f'seq4x2_{rep}'] = timed(seq)
        out[f'conc4x2_{rep}'] = timed(conc)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
