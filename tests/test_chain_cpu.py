"""The data side of the drop-in chain from the seed, against the oracle replayed
independently (nothing copied from the product): C1 = the bundled ml-100k atomic
files -> Config -> init_seed(2020) -> create_dataset -> data_preparation -> BPR.

Oracle (oracle/cpu_ref.py): atomic-file read + item filter + factorize remap
(dataset.py:844-928), the RO torch.randperm and the grouped ratio split
(dataset.py:1258-1315, 1377-1413), the sampler's numpy shuffle
(sampler.py:45-57), nn.Embedding + xavier_normal_ user then item (bpr.py:33-45,
init.py:15-31). The eval loaders sort their split by user in place with a stable
sort (general_dataloader.py:161-166, interaction.py:278-316), as the reference."""
import os

import numpy as np
import torch

from conftest import ROOT
from oracle import cpu_ref

DATA = os.path.join(ROOT, 'dataset')


def _product_c1():
    from recbole.config import Config
    from recbole.data import create_dataset, data_preparation
    from recbole.utils import get_model, init_seed
    config = Config(model='BPR', dataset='ml-100k',
                    config_dict={'data_path': DATA, 'use_gpu': False, 'state': 'ERROR'})
    init_seed(config['seed'], config['reproducibility'])
    ds = create_dataset(config)
    train, valid, test = data_preparation(config, ds)
    model = get_model('BPR')(config, train)
    return config, train, valid, test, model


def test_c1_ml100k_chain_from_seed():
    config, train, valid, test, model = _product_c1()
    after = torch.get_rng_state()

    u, i, nu, ni = cpu_ref.load_ml100k(os.path.join(DATA, 'ml-100k'))
    assert (len(u), nu, ni) == (99991, 944, 1682)
    torch.manual_seed(2020)
    np.random.seed(2020)
    parts = cpu_ref.ro_rs_split(u, (0.8, 0.1, 0.1))
    assert [len(p) for p in parts] == [80799, 9596, 9596]
    rl = cpu_ref.random_list_uniform(ni)
    ref = cpu_ref.BPRCPU(nu, ni, 64)

    for k, (p, data) in enumerate(zip(parts, (train, valid, test))):
        if k:                                           # eval loaders: stable sort by user
            p = p[np.argsort(u[p], kind='stable')]
        f = data.dataset.inter_feat
        assert np.array_equal(f['user_id'].numpy(), u[p]), k
        assert np.array_equal(f['item_id'].numpy(), i[p]), k
    assert np.array_equal(train.sampler.random_list, rl)
    assert torch.equal(model.user_embedding.weight.detach(), ref.user_embedding.weight.detach())
    assert torch.equal(model.item_embedding.weight.detach(), ref.item_embedding.weight.detach())
    assert torch.equal(after, torch.get_rng_state())    # next draw = epoch 0's randperm
    assert len(train) == 40 and train.step == 2048 and train.times == 1


def test_oracle_split_restatement_matches_loop_form():
    """The vectorised ro_rs_split against the reference's loops as written
    (dict of groups in first-appearance order, dataset.py:1249-1256, 1296-1303)."""
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 500):
        users = rng.integers(1, 12, n)
        torch.manual_seed(5)
        got = cpu_ref.ro_rs_split(users, (0.8, 0.1, 0.1))
        torch.manual_seed(5)
        perm = torch.randperm(n).numpy()
        groups = {}
        for pos, key in enumerate(users[perm]):
            groups.setdefault(key, []).append(pos)
        want = [[], [], []]
        for g in groups.values():
            ids = list(cpu_ref.calcu_split_ids(len(g), [0.8, 0.1, 0.1]))
            for part, s, e in zip(want, [0] + ids, ids + [len(g)]):
                part.extend(g[s:e])
        for a, b in zip(got, want):
            assert a.tolist() == perm[np.asarray(b, dtype=np.int64)].tolist()


def test_oracle_factorize_is_first_appearance():
    ids, n = cpu_ref.factorize(['b', 'a', 'b', 'c', 'a'])
    assert ids.tolist() == [1, 2, 1, 3, 2] and n == 4
