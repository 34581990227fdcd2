"""Breakdown of the C2 full-sort evaluation (bench.py's `eval` line): K6 launch(es),
flags to the host, metric reduction — wall time of each part, synchronized."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from recbole_amd import ops
    from recbole_amd.evaluator import TopKEvaluator
    from recbole_amd.trainer.fused import fused_full_sort_eval
    dev = torch.device('cuda', 0)
    config, train, test, model, opt, step = bench.build_workload(dev)
    ev = TopKEvaluator(config, ['recall', 'mrr', 'ndcg', 'hit', 'precision'])
    fused_full_sort_eval(model, test, ev)
    torch.cuda.synchronize()
    for _ in range(3):
        t = {}
        t0 = time.perf_counter()
        K = max(ev.topk)
        uids, hp, hc, pp, pc = test.device_csr(dev)
        EI = model.fused_item_table().contiguous()
        Uq = model.fused_user_vectors(uids).contiguous()
        torch.cuda.synchronize()
        t['prep'] = time.perf_counter() - t0
        t0 = time.perf_counter()
        o = ops.fullsort_topk(Uq, EI, K, hist_ptr=hp, hist_cols=hc, pos_ptr=pp, pos_cols=pc)
        torch.cuda.synchronize()
        t['k6'] = time.perf_counter() - t0
        t0 = time.perf_counter()
        pos_idx = o['pos_flags'].cpu().numpy().astype(bool)
        t['d2h'] = time.perf_counter() - t0
        t0 = time.perf_counter()
        pl = test.get_pos_len_list()
        t['pos_len'] = time.perf_counter() - t0
        t0 = time.perf_counter()
        ev.evaluate_pos_idx(pos_idx, pl)
        t['metrics'] = time.perf_counter() - t0
        t0 = time.perf_counter()
        fused_full_sort_eval(model, test, ev)
        torch.cuda.synchronize()
        t['total'] = time.perf_counter() - t0
        print({k: round(v * 1e3, 2) for k, v in t.items()}, 'ms', flush=True)


if __name__ == '__main__':
    main()
