"""K36 (csrc/step.hip chunk_group_kernel, mirec_chunk_group): a chunk's groupings, K35
records and look-ahead lists in ONE launch — bit for bit against the launches it
replaces on the C2 path: the K2 LDS radix sort (mirec_segment_sort_batched: perm, uniq,
seg, n_uniq per batch), mirec_step_records (row / share / contribution records) and
mirec_uniq_ahead_diff (uniq(b+1) minus uniq(b), ascending).

Cases: the C2 shape (512 positives, 4 negatives, 138,494 x 26,745 rows) with Zipf
positives and uniform negatives; one-batch and many-batch chunks; T = 1 and 6; a ragged
batch (37 positives); duplicate-heavy batches (items from 3 ids: more shares than the
256 a batch deals out); user keys with repeats; the shape bounds (Bc = 2,048 at T = 1:
4,096 item slots) and a shape outside them (reported, nothing written)."""
import numpy as np
import pytest
import torch

from recbole_amd import ops

pytestmark = pytest.mark.gpu

NU, NI = 138494, 26745


def _keys(dev, nb, Bc, T, gen, few=0, dup_users=False):
    KI = (1 + T) * Bc
    if dup_users:
        users = torch.randint(1, 40, (nb * Bc,), generator=gen)
    else:
        users = torch.randint(1, NU, (nb * Bc,), generator=gen)
    items = torch.empty(nb, 1 + T, Bc, dtype=torch.int64)
    if few:
        items[:] = torch.randint(1, few + 1, (nb, 1 + T, Bc), generator=gen)
    else:
        z = torch.distributions.Categorical(probs=1.0 / torch.arange(1, NI, dtype=torch.float64))
        torch.manual_seed(int(torch.randint(0, 1 << 30, (1,), generator=gen)))
        items[:, 0, :] = z.sample((nb, Bc)) + 1
        items[:, 1:, :] = torch.randint(1, NI, (nb, T, Bc), generator=gen)
    return users.to(dev), items.reshape(nb * KI).to(dev)


def _outs(dev, nb, Bc, T):
    KI = (1 + T) * Bc
    z = lambda n: torch.zeros(n, dtype=torch.int32, device=dev)
    o = {}
    for tag, per in (('u', Bc), ('i', KI)):
        o[f'{tag}_perm'], o[f'{tag}_uniq'] = z(nb * per), z(nb * per)
        o[f'{tag}_seg'], o[f'{tag}_nu'] = z(nb * (per + 1)), z(nb)
        o[f'{tag}_rec'], o[f'{tag}_crec'] = z(nb * ops.step_record_ints(per)), z(nb * per * 8)
        o[f'{tag}_ahead'], o[f'{tag}_nah'] = z(nb * per), z(nb)
    return o


def _reference(users, items, nb, Bc, T, o):
    """The launches K36 replaces, on the same keys."""
    KI = (1 + T) * Bc
    from types import SimpleNamespace
    for tag, keys, per, space in (('u', users, Bc, NU), ('i', items, KI, NI)):
        ops.segment_sort_batched(keys, per, space, o[f'{tag}_perm'], o[f'{tag}_uniq'],
                                 o[f'{tag}_seg'], o[f'{tag}_nu'])
        ops.uniq_ahead_diff(o[f'{tag}_uniq'], o[f'{tag}_nu'], per, nb, o[f'{tag}_ahead'],
                            o[f'{tag}_nah'])
    g = {t: SimpleNamespace(perm=o[f'{t}_perm'], uniq=o[f'{t}_uniq'], seg=o[f'{t}_seg'],
                            n_uniq=o[f'{t}_nu']) for t in 'ui'}
    ops.step_records(users, items, nb, Bc, T, NU, NI, g['u'], g['i'],
                     out=[o[k] for k in ('u_rec', 'u_crec', 'i_rec', 'i_crec')])


def _valid_mask(o, nb, Bc, T):
    """Per output, the positions both paths define."""
    KI = (1 + T) * Bc
    masks = {}
    for tag, per in (('u', Bc), ('i', KI)):
        nu = o[f'{tag}_nu'].cpu().numpy()
        nah = o[f'{tag}_nah'].cpu().numpy()
        ri = ops.step_record_ints(per)
        rec = np.zeros(nb * ri, bool)
        rec_ints = o[f'{tag}_rec'].cpu().numpy()
        ah = np.zeros(nb * per, bool)
        for b in range(nb):
            base = b * ri
            rec[base:base + nu[b] * 20] = True                      # row records (kRowRec 20)
            ntask = rec_ints[base + per * 20 + 256 * 24]            # task count
            rec[base + per * 20:base + per * 20 + ntask * 24] = True
            rec[base + per * 20 + 256 * 24] = True
            ah[b * per:b * per + nah[b]] = True
        useg = np.zeros(nb * (per + 1), bool)
        uq = np.zeros(nb * per, bool)
        for b in range(nb):
            useg[b * (per + 1):b * (per + 1) + nu[b] + 1] = True
            uq[b * per:b * per + nu[b]] = True
        masks.update({f'{tag}_rec': rec, f'{tag}_ahead': ah, f'{tag}_seg': useg,
                      f'{tag}_uniq': uq})
    return masks


@pytest.mark.parametrize('nb,Bc,T,few,dup', [(1, 512, 4, 0, False), (4, 512, 4, 0, False),
                                             (9, 512, 4, 0, True), (3, 37, 4, 0, False),
                                             (2, 512, 1, 0, False), (3, 300, 6, 0, False),
                                             (3, 512, 4, 3, False), (2, 2048, 1, 0, False),
                                             (2, 512, 4, 5, True)])
def test_chunk_group_equals_sort_records_ahead(dev, nb, Bc, T, few, dup):
    gen = torch.Generator().manual_seed(nb * 1000 + Bc + T + few)
    users, items = _keys(dev, nb, Bc, T, gen, few, dup)
    ref, got = _outs(dev, nb, Bc, T), _outs(dev, nb, Bc, T)
    _reference(users, items, nb, Bc, T, ref)
    assert ops.chunk_group(users, items, nb, Bc, T, NU, NI, got)
    torch.cuda.synchronize()
    masks = _valid_mask(ref, nb, Bc, T)
    for k in ref:
        a, b = ref[k].cpu().numpy(), got[k].cpu().numpy()
        m = masks.get(k)
        if m is not None:
            a, b = a[m], b[m]
        assert np.array_equal(a, b), (k, np.flatnonzero(a != b)[:10])


def test_chunk_group_without_records_or_lists(dev):
    """The K3 + K5 path's form: groupings only (records and lists NULL), and the
    look-ahead lists without records."""
    gen = torch.Generator().manual_seed(5)
    nb, Bc, T = 3, 512, 4
    users, items = _keys(dev, nb, Bc, T, gen)
    ref = _outs(dev, nb, Bc, T)
    _reference(users, items, nb, Bc, T, ref)
    for records, ahead in ((False, False), (False, True)):
        got = _outs(dev, nb, Bc, T)
        assert ops.chunk_group(users, items, nb, Bc, T, NU, NI, got, records=records, ahead=ahead)
        masks = _valid_mask(ref, nb, Bc, T)
        keys = ['u_perm', 'u_uniq', 'u_seg', 'u_nu', 'i_perm', 'i_uniq', 'i_seg', 'i_nu']
        if ahead:
            keys += ['u_ahead', 'u_nah', 'i_ahead', 'i_nah']
        for k in keys:
            a, b = ref[k].cpu().numpy(), got[k].cpu().numpy()
            m = masks.get(k)
            if m is not None:
                a, b = a[m], b[m]
            assert np.array_equal(a, b), k
        if not records:
            assert int(got['u_rec'].abs().sum()) == 0 and int(got['i_crec'].abs().sum()) == 0


def test_chunk_group_declines_outside_its_shapes(dev):
    """(1+T)*Bc > 4,096 item slots: returns False and writes nothing."""
    gen = torch.Generator().manual_seed(6)
    nb, Bc, T = 1, 1024, 4
    users, items = _keys(dev, nb, Bc, T, gen)
    got = _outs(dev, nb, Bc, T)
    assert not ops.chunk_group(users, items, nb, Bc, T, NU, NI, got)
    torch.cuda.synchronize()
    assert all(int(v.abs().sum()) == 0 for v in got.values())
