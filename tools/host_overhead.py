"""Host-side cost of one training step (enqueue only) vs the synchronized step time."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _transport(dev):
    """SS_ENGINE_GENERAL=xgmi: the N>1 path through a size-1 mailbox arena."""
    if os.environ.get("SS_ENGINE_GENERAL") == "xgmi":
        from swiftsnails_amd.parallel.xgmi import XgmiTransport

        return XgmiTransport(0, 1, dev, None)
    return None


def _worker(model, dev):
    from swiftsnails_amd.parallel.engine import PSEngine

    if model == "lr":
        from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table

        data = CtrSynth()
        table = make_lr_table(data.num_features, device=dev)
        eng = PSEngine(table, _transport(dev), max_keys=data.batch_size * data.num_fields, dim=1,
                       device=dev)
        return SparseLRWorker(eng, data)
    from swiftsnails_amd.models.word2vec import W2VSynth, Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.table import HbmTable

    data = W2VSynth(mode="pairs" if model == "w2v_pairs" else "window")
    opt, init = make_w2v_table_args(128)
    table = HbmTable(128, int(2 * data.vocab / 0.5) + 1024, optimizer=opt, init=init, device=dev)
    eng = PSEngine(table, _transport(dev), max_keys=data.n_keys, dim=128, device=dev)
    return Word2VecWorker(eng, data)


def main():
    """python tools/host_overhead.py [lr|w2v|w2v_pairs]  (SS_ENGINE_GENERAL=xgmi: N>1 path)"""
    dev = torch.device("cuda", 0)
    w = _worker(sys.argv[1] if len(sys.argv) > 1 else "lr", dev)
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
    for _ in range(500):
        w.step()
    pr.disable()
    torch.cuda.synchronize()
    # 500 steps: 1 ms of tottime = 2 us per step
    pstats.Stats(pr).sort_stats("tottime").print_stats(40)


if __name__ == "__main__":
    main()
