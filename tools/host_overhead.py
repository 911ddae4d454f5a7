"""Host-side cost of one training step (enqueue only) vs the synchronized step time."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
    from swiftsnails_amd.parallel.engine import PSEngine

    dev = torch.device("cuda", 0)
    data = CtrSynth()
    table = make_lr_table(data.num_features, device=dev)
    eng = PSEngine(table, None, max_keys=data.batch_size * data.num_fields, dim=1, device=dev)
    w = SparseLRWorker(eng, data)
    for _ in range(10):
        w.step()
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        w.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e6 * (t1 - t0) / n:.1f} us/step, wall {1e6 * (t2 - t0) / n:.1f} us/step")
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        w.step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
