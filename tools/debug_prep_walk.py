"""Debug (GPU): the C2 chunk-0 walk through (a) ops.sample_walk one batch at a
time, (b) one multi-batch launch, (c) the fused step's native chunk preparation
— each against the oracle's C walk on the same keys."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from oracle import cpu_ref
    from recbole_amd import ops
    dev = torch.device('cuda', 0)
    config, train, test, model, opt, step = bench.build_workload(dev)
    samp = train.sampler
    B, T, nb = step.B, step.times, 8
    step.RAMP = ()
    step.begin_epoch(cuts=(nb,), hold_prep_from=0)     # nothing prepared yet
    users = step._users[:nb * B].clone()
    ptr, cols = samp.used_csr['train']
    rl = np.asarray(samp.random_list)
    exp, pr = [], 0
    for b in range(nb):
        o, pr = cpu_ref.c_sample_walk(rl, pr, users[b * B:(b + 1) * B].cpu().numpy(), T, ptr, cols,
                                      step.nU, True)
        exp.append(o)
    exp = np.stack(exp)
    rl_d, pr_d, up, uc, bits, n_bits, reject, status = samp.walk_args(dev)
    # (a) batch at a time
    pr_d.zero_()
    got_a = np.stack([ops.sample_walk(rl_d, pr_d, users[b * B:(b + 1) * B], T, up, uc, step.nU, True,
                                      used_bits=bits, n_bits=n_bits).cpu().numpy()
                      for b in range(nb)])
    # (b) one launch
    pr_d.zero_()
    out = torch.empty(nb * B * T, dtype=torch.int64, device=dev)
    ops.sample_walk(rl_d, pr_d, users, T, up, uc, step.nU, True, batch_keys=B, n_batches=nb,
                    out=out, used_bits=bits, n_bits=n_bits)
    got_b = out.view(nb, B * T).cpu().numpy()
    # (c) the fused step's chunk preparation
    pr_d.zero_()
    torch.cuda.synchronize()
    step.release_prep()
    step._issue_prep()
    torch.cuda.synchronize()
    KI = (1 + T) * B
    got_c = step.slots[0].item_keys[:nb * KI].view(nb, KI)[:, B:].cpu().numpy()
    for name, g in (('a', got_a), ('b', got_b), ('c', got_c)):
        bad = np.argwhere(g != exp)
        print(name, 'mismatches', len(bad), bad[:6].tolist(), flush=True)


if __name__ == '__main__' and len(sys.argv) == 1:
    main()


def chain():
    """The chain test's first part with a snapshot of the walk before training."""
    import bench
    from oracle import cpu_ref
    dev = torch.device('cuda', 0)
    config, train, test, model, opt, step = bench.build_workload(dev)
    C, B, T = step.C, step.B, step.times
    KI = (1 + T) * B
    step.RAMP = ()
    print('pr after build:', train.sampler.random_pr, flush=True)
    step.begin_epoch(cuts=(C,), hold_prep_from=0)
    torch.cuda.synchronize()
    print('pr after begin_epoch (held):', train.sampler.random_pr, flush=True)
    step.release_prep()
    step._issue_prep()
    torch.cuda.synchronize()
    print('pr after chunk 0 prep:', train.sampler.random_pr, flush=True)
    before = step.slots[0].item_keys[:C * KI].view(C, KI)[:, B:].cpu().numpy().copy()
    users = step._users[:C * B].cpu().numpy()
    samp = train.sampler
    ptr, cols = samp.used_csr['train']
    rl = np.asarray(samp.random_list)
    exp, pr = [], 0
    for b in range(C):
        o, pr = cpu_ref.c_sample_walk(rl, pr, users[b * B:(b + 1) * B], T, ptr, cols, step.nU, True)
        exp.append(o)
    exp = np.stack(exp)
    print('walk before training vs oracle:', int((before != exp).sum()), flush=True)
    step.run_batches(0, C)
    step.end_epoch(C)
    after = step.slots[0].item_keys[:C * KI].view(C, KI)[:, B:].cpu().numpy()
    print('after training vs before:', int((after != before).sum()),
          'vs oracle:', int((after != exp).sum()), flush=True)


if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'chain':
    chain()
