"""Debug: per-row comparison of the fused uni-N evaluation (K9c ranks) with the
generic loader + predict + flip/topk sequence on the SASRec test pipeline."""
import pathlib, sys, tempfile
sys.path.insert(0, '.')
import numpy as np
import torch
from tests.test_gpu_sasrec import _pipeline
from recbole_amd._native import lib, ptr, stream_handle

tmp = pathlib.Path(tempfile.mkdtemp())
config, train, valid, test, model = _pipeline(tmp)
model.eval()
dev = config['device']
s = valid.sampler
s.to_device(dev)
L = s.random_list_length
rows = 0
bad = 0
with torch.no_grad():
    for start in range(0, valid.pr_end, valid.step):
        pr0 = s.random_pr
        valid.pr = start
        b = valid._next_batch_data()
        gen_items = b['item_id'].view(-1, 1001)
        gen_scores = model.predict(b.to(dev)).view(-1, 1001)
        flip = torch.flip(gen_scores, dims=[-1])
        _, ti = torch.topk(flip, 10)
        gpos = [(int((ti[r] >= 1000).nonzero()[0]) if (ti[r] >= 1000).any() else -1)
                for r in range(ti.shape[0])]
        s.random_pr = pr0
        inter = valid.augmentation(slice(start, start + valid.step)).to(dev)
        n, m = inter['user_id'].numel(), valid.neg_sample_by
        idx = (s._pr_dev + torch.arange(n * m, device=dev)) % L
        neg = s._rl_dev[idx].to(torch.int64)
        s._pr_dev.copy_((s._pr_dev + n * m) % L)
        S = model.fused_query_vectors(inter).contiguous()
        rank = torch.empty(n, dtype=torch.int32, device=dev)
        pos = inter['item_id'].contiguous()
        E = model.item_embedding.weight.detach()
        lib().mirec_rank_of_pos_f32(ptr(S), ptr(E), E.shape[0], E.shape[1], ptr(pos), ptr(neg),
                                    n, m, ptr(rank), stream_handle())
        fr = rank.tolist()
        for r in range(n):
            f = fr[r] if fr[r] < 10 else -1
            if f != gpos[r] or not torch.equal(neg.view(n, m)[r].cpu(), gen_items[r, 1:].cpu()):
                bad += 1
                g = gen_scores[r]
                print('row', rows + r, 'fused', fr[r], 'generic pos', gpos[r],
                      'gt/ge', (g[1:] > g[0]).sum().item(), (g[1:] >= g[0]).sum().item(),
                      'negs equal', torch.equal(neg.view(n, m)[r].cpu(), gen_items[r, 1:].cpu()))
        rows += n
print('rows', rows, 'mismatches', bad)
