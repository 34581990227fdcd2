"""Atomic-file dataset (mirror of the parts of recbole/data/dataset/dataset.py
the general-recommendation path uses).

Pipeline, in the reference's order (dataset.py:100-157, 160-178):
  load .inter/.user/.item (pandas, `field:type` headers, load_col/unload_col)
  -> filter NaN ids -> remove duplicates -> filter by value
  -> drop inters whose user/item is missing from .user/.item
  -> k-core / inter-num filter -> reset index
  -> remap every token field with pandas.factorize (ids by first appearance,
     0 = [PAD]; inter column first, then the feature file) (dataset.py:878-928)
  -> order user/item feats by id, fill NaN, min-max normalise
  -> build(): to Interaction, RO shuffle (torch.randperm) or TO sort, then
     ratio split grouped by user (_calcu_split_ids) or leave-one-out
     (dataset.py:1249-1413).
Row-id parity with the reference depends on this order; it is pinned by the
reference's own dataset tests (tests/test_dataset_pipeline.py).
"""
from __future__ import annotations

import copy
import os
from collections import Counter
from logging import getLogger

import numpy as np
import pandas as pd
import torch

from recbole_amd.data.interaction import Interaction
from recbole_amd.utils import FeatureSource, FeatureType


def _stable_order(keys):
    """np.argsort(keys, kind='stable'); a counting sort (native, O(n)) for
    non-negative integer keys of a moderate range (remapped ids)."""
    keys = np.asarray(keys)
    if (keys.dtype.kind in 'iu' and len(keys) > 4096 and keys.min() >= 0
            and keys.max() < 4 * len(keys) + (1 << 16)):
        from recbole_amd import ops
        return ops.host_counting_order(keys, int(keys.max()) + 1)
    return np.argsort(keys, kind='stable')


def _group_layout(keys):
    """Rows grouped by key: (rows in (group first-appearance, position) order, each
    row's group (first-appearance rank), position in its group, group sizes in
    first-appearance order)."""
    order = _stable_order(keys)
    sk = keys[order]
    starts = np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]])
    tot = np.diff(np.r_[starts, len(sk)]).astype(np.int64)
    gperm = np.argsort(order[starts], kind='stable')          # groups by first appearance
    grank = np.empty(len(tot), dtype=np.int64)
    grank[gperm] = np.arange(len(tot))
    grp = np.repeat(np.arange(len(tot)), tot)
    pos = np.arange(len(sk)) - np.repeat(starts, tot)
    goff = np.empty(len(tot), dtype=np.int64)
    goff[gperm] = np.r_[0, np.cumsum(tot[gperm])[:-1]]
    newpos = goff[grp] + pos
    rows = np.empty(len(sk), dtype=np.int64)
    rows[newpos] = order
    g_of = np.empty(len(sk), dtype=np.int64)
    g_of[newpos] = grank[grp]
    p_of = np.empty(len(sk), dtype=np.int64)
    p_of[newpos] = pos
    return rows, g_of, p_of, tot[gperm]


def _grouped_leave_one_out(keys, leave_one_num):
    """leave_one_out (dataset.py:1317-1337), vectorised: per group (first-appearance
    order) legal = min(leave_one_num, size - 1); the first size - legal rows go to
    part 0 and the last `legal` rows to parts P - legal .. P - 1 (P = leave_one_num + 1),
    in row order."""
    keys = np.asarray(keys)
    P = leave_one_num + 1
    if len(keys) == 0:
        return [np.zeros(0, dtype=np.int64) for _ in range(P)]
    rows, g, pos, sizes = _group_layout(keys)
    size = sizes[g]
    legal = np.minimum(leave_one_num, size - 1)
    pr = size - legal
    part = np.where(pos < pr, 0, P - legal + (pos - pr))
    return [rows[part == q] for q in range(P)]


def _grouped_ratio_split(keys, ratios):
    """split_by_ratio with group_by (dataset.py:1281-1315), vectorised: groups in
    first-appearance order, rows of a group in their current order, and group g's
    part sizes from _calcu_split_ids(len(g), ratios) — the same float64 products,
    truncations and remainder rule, evaluated for every group at once. Returns the
    row indices of each part, groups concatenated in first-appearance order."""
    keys = np.asarray(keys)
    R = len(ratios)
    if len(keys) == 0:
        return [np.zeros(0, dtype=np.int64) for _ in range(R)]
    order = _stable_order(keys)
    sk = keys[order]
    starts = np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]])
    sizes = np.diff(np.r_[starts, len(sk)])
    gperm = np.argsort(order[starts], kind='stable')          # groups by first appearance
    # part sizes per group (_calcu_split_ids over every group)
    tot = sizes.astype(np.int64)
    totf = tot.astype(np.float64)
    cnt = [None] + [np.floor(ratios[i] * totf).astype(np.int64) for i in range(1, R)]
    cnt[0] = tot - (sum(cnt[1:]) if R > 1 else 0)
    done = np.zeros(len(tot), dtype=bool)
    for i in range(1, R):
        done |= cnt[0] <= 1
        x = ratios[-i] * totf
        bump = ~done & (x > 0) & (x < 1)
        cnt[-i] = cnt[-i] + bump
        cnt[0] = cnt[0] - bump
    # every row's position inside its group and its part
    grp = np.repeat(np.arange(len(tot)), tot)
    pos = np.arange(len(sk)) - np.repeat(starts, tot)
    part = np.zeros(len(sk), dtype=np.int64)
    edge = np.zeros(len(tot), dtype=np.int64)
    for i in range(R - 1):
        edge = edge + cnt[i]
        part += pos >= edge[grp]
    # rows in (group first-appearance, position) order
    goff = np.empty(len(tot), dtype=np.int64)
    goff[gperm] = np.r_[0, np.cumsum(tot[gperm])[:-1]]
    rows = np.empty(len(sk), dtype=np.int64)
    newpos = goff[grp] + pos
    rows[newpos] = order
    part_sorted = np.empty(len(sk), dtype=np.int64)
    part_sorted[newpos] = part
    return [rows[part_sorted == p] for p in range(R)]


def _counts(col):
    """Counter of a column's values (same keys and counts as Counter(col.values))."""
    vc = col.value_counts(dropna=True, sort=False)
    vc = vc[vc.values > 0]                      # a Categorical lists unseen categories too
    return Counter(dict(zip(vc.index.tolist(), vc.values.tolist())))


def _factorize(pieces):
    """pd.factorize(np.concatenate(pieces)) for pieces that are object arrays or
    pandas Categoricals: codes in order of first appearance over the concatenation
    (missing -> -1) and the distinct values in that order. Categorical pieces are
    resolved through their integer codes (the string work is per distinct value)."""
    ids, order = {}, []
    out = []
    for t in pieces:
        if isinstance(t, pd.Categorical):
            codes = t.codes.astype(np.int64)
            cats = np.asarray(t.categories, dtype=object)
        else:
            c, u = pd.factorize(np.asarray(t, dtype=object))
            codes, cats = c.astype(np.int64), np.asarray(u, dtype=object)
        seen = pd.unique(codes[codes >= 0])      # this piece's first-appearance order
        lut = np.full(len(cats) + 1, -1, dtype=np.int64)
        for lc in seen.tolist():
            tok = cats[lc]
            g = ids.get(tok)
            if g is None:
                g = ids[tok] = len(order)
                order.append(tok)
            lut[lc] = g
        out.append(lut[codes])                   # code -1 reads lut[-1] = -1
    new_ids = np.concatenate(out) if out else np.zeros(0, dtype=np.int64)
    return new_ids, np.array(order, dtype=object)


def _pandas_na_tokens():
    """The strings pd.read_csv reads as missing by default (its na_values); Arrow's
    own default list lacks 'None' and '<NA>'."""
    try:
        from pandas._libs.parsers import STR_NA_VALUES
        return sorted(STR_NA_VALUES)
    except ImportError:                          # the documented pandas default list
        return ['', '#N/A', '#N/A N/A', '#NA', '-1.#IND', '-1.#QNAN', '-NaN', '-nan', '1.#IND',
                '1.#QNAN', '<NA>', 'N/A', 'NA', 'NULL', 'NaN', 'None', 'n/a', 'nan', 'null']


_PANDAS_NA_TOKENS = _pandas_na_tokens()


def _read_atomic(filepath, sep, usecols, dtype, cat_cols=()):
    """pd.read_csv(filepath, delimiter=sep, usecols=usecols, dtype=dtype) as the
    reference reads an atomic file (dataset.py:342-408), parsed by Arrow's
    multi-threaded CSV reader: token columns as strings (pandas' missing-value tokens,
    quoted or not, -> missing, like its NaN), float columns as float64, then the same pandas frame (object
    columns of str). Float fields are parsed correctly rounded (pandas' default
    parser may differ in the last bit for inputs of more than ~15 significant digits;
    atomic-file ratings, timestamps and prices are exact either way). Columns in
    `cat_cols` (single-token fields) come back as pandas Categoricals of the same
    strings: the filters and the remap then work on integer codes (_factorize)."""
    try:
        import pyarrow as pa
        import pyarrow.csv as pacsv
    except ImportError:                         # plain pandas when Arrow is absent
        return pd.read_csv(filepath, delimiter=sep, usecols=usecols, dtype=dtype)
    types = {c: (pa.float64() if dtype[c] is np.float64 else pa.string()) for c in usecols}
    try:
        tb = pacsv.read_csv(
            filepath, parse_options=pacsv.ParseOptions(delimiter=sep),
            convert_options=pacsv.ConvertOptions(column_types=types,
                                                 include_columns=list(usecols),
                                                 null_values=_PANDAS_NA_TOKENS,
                                                 strings_can_be_null=True,
                                                 quoted_strings_can_be_null=True))
    except pa.ArrowInvalid:
        # ragged rows (pandas fills missing trailing fields with NaN; Arrow refuses)
        return pd.read_csv(filepath, delimiter=sep, usecols=usecols, dtype=dtype)
    out = {}
    for c in usecols:
        col = tb.column(c)
        if dtype[c] is np.float64:
            out[c] = col.to_numpy().astype(np.float64, copy=False)
        elif c in cat_cols:                     # codes + distinct strings; null -> code -1
            enc = col.combine_chunks().dictionary_encode()
            codes = enc.indices.fill_null(-1).to_numpy(zero_copy_only=False).astype(np.int32)
            out[c] = pd.Categorical.from_codes(
                codes, categories=pd.Index(enc.dictionary.to_pylist(), dtype=object))
        else:                                   # object array of str / NaN like pandas
            v = col.to_pandas(types_mapper=None).to_numpy(dtype=object)
            if col.null_count:
                v[pd.isnull(v)] = np.nan
            out[c] = v
    return pd.DataFrame(out, columns=list(usecols))


class Dataset(object):

    @classmethod
    def from_interactions(cls, config, user_ids, item_ids, n_users, n_items, timestamps=None):
        """In-memory dataset of already-remapped ids (1..n-1; 0 = [PAD]), e.g. the
        synthetic benchmark workloads, without writing atomic files. Same
        downstream behaviour as a loaded dataset (build/split/loaders)."""
        self = cls.__new__(cls)
        self.config = config
        self.dataset_name = config['dataset']
        self.logger = getLogger()
        self.dataset_path = config['data_path']
        self.uid_field = config['USER_ID_FIELD']
        self.iid_field = config['ITEM_ID_FIELD']
        self.label_field = config['LABEL_FIELD']
        self.time_field = config['TIME_FIELD']
        self.benchmark_filename_list = None
        self.file_size_list = None
        self.field2type = {self.uid_field: FeatureType.TOKEN, self.iid_field: FeatureType.TOKEN}
        self.field2source = {self.uid_field: FeatureSource.USER_ID,
                             self.iid_field: FeatureSource.ITEM_ID}
        self.field2seqlen = {self.uid_field: 1, self.iid_field: 1}
        self.field2id_token = {self.uid_field: np.arange(n_users).astype(str),
                               self.iid_field: np.arange(n_items).astype(str)}
        self.field2id_token[self.uid_field][0] = '[PAD]'
        self.field2id_token[self.iid_field][0] = '[PAD]'
        self.field2token_id = {}
        cols = {self.uid_field: torch.as_tensor(np.asarray(user_ids, dtype=np.int64)),
                self.iid_field: torch.as_tensor(np.asarray(item_ids, dtype=np.int64))}
        if timestamps is not None:
            self.field2type[self.time_field] = FeatureType.FLOAT
            self.field2source[self.time_field] = FeatureSource.INTERACTION
            self.field2seqlen[self.time_field] = 1
            cols[self.time_field] = torch.as_tensor(np.asarray(timestamps, dtype=np.float32))
        self.inter_feat = Interaction(cols)
        self.user_feat = None
        self.item_feat = None
        self.feat_name_list = ['inter_feat']
        return self

    def __init__(self, config):
        self.config = config
        self.dataset_name = config['dataset']
        self.logger = getLogger()
        self.dataset_path = config['data_path']
        self.field2type, self.field2source = {}, {}
        self.field2id_token, self.field2token_id = {}, {}
        self.field2seqlen = dict(config['seq_len'] or {})
        self.uid_field = config['USER_ID_FIELD']
        self.iid_field = config['ITEM_ID_FIELD']
        self.label_field = config['LABEL_FIELD']
        self.time_field = config['TIME_FIELD']
        if (self.uid_field is None) ^ (self.iid_field is None):
            raise ValueError('USER_ID_FIELD and ITEM_ID_FIELD need to be set at the same time '
                             'or not set at the same time.')
        self.benchmark_filename_list = config['benchmark_filename']
        self._load_data(self.dataset_name, self.dataset_path)
        self.feat_name_list = [f for f in ['inter_feat', 'user_feat', 'item_feat']
                               if getattr(self, f, None) is not None]
        if self.benchmark_filename_list is None:
            self._data_filtering()
        self._remap_ID_all()
        self._user_item_feat_preparation()
        self._fill_nan()
        self._set_label_by_threshold()
        self._normalize()

    # ------------------------------------------------------------------ loading
    def _load_data(self, token, path):
        if self.benchmark_filename_list is None:
            self.inter_feat = self._load_feat(os.path.join(path, f'{token}.inter'),
                                              FeatureSource.INTERACTION)
            self.file_size_list = None
        else:
            sub = []
            for fn in self.benchmark_filename_list:
                sub.append(self._load_feat(os.path.join(path, f'{token}.{fn}.inter'),
                                           FeatureSource.INTERACTION))
            self.file_size_list = [len(s) for s in sub]
            self.inter_feat = pd.concat(sub, ignore_index=True)
        if self.inter_feat is None:
            raise ValueError(f'File {os.path.join(path, token + ".inter")} not exist.')
        self.user_feat = self._load_feat_if_exists(os.path.join(path, f'{token}.user'),
                                                   FeatureSource.USER, self.uid_field)
        self.item_feat = self._load_feat_if_exists(os.path.join(path, f'{token}.item'),
                                                   FeatureSource.ITEM, self.iid_field)

    def _load_feat_if_exists(self, filepath, source, field):
        if not os.path.isfile(filepath):
            return None
        feat = self._load_feat(filepath, source)
        if feat is not None and field is not None and field not in feat:
            raise ValueError(f'{field} must be loaded if {source.value}_feat is loaded.')
        if feat is not None and field in self.field2source:
            self.field2source[field] = FeatureSource(source.value + '_id')
        return feat

    def _get_load_and_unload_col(self, source):
        src = source.value if isinstance(source, FeatureSource) else source
        lc, uc = self.config['load_col'], self.config['unload_col']
        load_col = None if lc is None else (set(lc[src]) if src in lc else set())
        unload_col = None if uc is None or src not in uc else set(uc[src])
        if load_col and unload_col:
            raise ValueError(f'load_col [{load_col}] and unload_col [{unload_col}] can not be '
                             f'set the same time.')
        return load_col, unload_col

    def _load_feat(self, filepath, source):
        if not os.path.isfile(filepath):
            return None
        load_col, unload_col = self._get_load_and_unload_col(source)
        if load_col == set():
            return None
        sep = self.config['field_separator']
        with open(filepath, 'r') as f:
            head = f.readline().rstrip('\n').rstrip('\r')
        columns, usecols, dtype = [], [], {}
        for field_type in head.split(sep):
            field, ftype = field_type.split(':')
            try:
                ftype = FeatureType(ftype)
            except ValueError:
                raise ValueError(f'Type {ftype} from field {field} is not supported.')
            if load_col is not None and field not in load_col:
                continue
            if unload_col is not None and field in unload_col:
                continue
            self.field2source[field] = source
            self.field2type[field] = ftype
            if not ftype.value.endswith('seq'):
                self.field2seqlen[field] = 1
            columns.append(field)
            usecols.append(field_type)
            dtype[field_type] = np.float64 if ftype == FeatureType.FLOAT else str
        if not columns:
            return None
        cats = {ft for ft, f in zip(usecols, columns) if self.field2type[f] == FeatureType.TOKEN}
        df = _read_atomic(filepath, sep, usecols, dtype, cats)
        df.columns = columns
        seq_sep = self.config['seq_separator']
        for field in columns:
            ftype = self.field2type[field]
            if not ftype.value.endswith('seq'):
                continue
            df[field] = df[field].fillna(value='')
            if ftype == FeatureType.TOKEN_SEQ:
                df[field] = [np.array(list(filter(None, s.split(seq_sep)))) for s in df[field].values]
            else:
                df[field] = [np.array(list(map(float, filter(None, s.split(seq_sep)))))
                             for s in df[field].values]
            self.field2seqlen[field] = max(map(len, df[field].values)) if len(df) else 0
        return df

    # ------------------------------------------------------------------ filtering
    def _data_filtering(self):
        self._filter_nan_user_or_item()
        self._remove_duplication()
        self._filter_by_field_value()
        self._filter_inter_by_user_or_item()
        self._filter_by_inter_num()
        self._reset_index()

    def _filter_nan_user_or_item(self):
        for field, name in [(self.uid_field, 'user'), (self.iid_field, 'item')]:
            feat = getattr(self, name + '_feat')
            if feat is not None:
                drop = feat.index[feat[field].isnull()]
                if len(drop):
                    feat.drop(drop, inplace=True)
            if field is not None:
                drop = self.inter_feat.index[self.inter_feat[field].isnull()]
                if len(drop):
                    self.inter_feat.drop(drop, inplace=True)

    def _remove_duplication(self):
        keep = self.config['rm_dup_inter']
        if keep is None:
            return
        if self.time_field in self.inter_feat:
            self.inter_feat.sort_values(by=[self.time_field], ascending=True, inplace=True,
                                        kind='stable')
        self.inter_feat.drop_duplicates(subset=[self.uid_field, self.iid_field], keep=keep,
                                        inplace=True)

    def _drop_by_value(self, val, cmp):
        if val is None:
            return []
        for field in val:
            if field not in self.field2type:
                raise ValueError(f'Field [{field}] not defined in dataset.')
            if self.field2type[field] not in {FeatureType.FLOAT, FeatureType.FLOAT_SEQ}:
                raise ValueError(f"Field [{field}] is not float-like field in dataset, "
                                 f"which can't be filter.")
            for fname in self.feat_name_list:
                feat = getattr(self, fname)
                if field in feat:
                    feat.drop(feat.index[cmp(feat[field].values, val[field])], inplace=True)
        return list(val)

    def _filter_by_field_value(self):
        self._drop_by_value(self.config['lowest_val'], lambda x, y: x < y)
        self._drop_by_value(self.config['highest_val'], lambda x, y: x > y)
        self._drop_by_value(self.config['equal_val'], lambda x, y: x != y)
        self._drop_by_value(self.config['not_equal_val'], lambda x, y: x == y)

    def _filter_inter_by_user_or_item(self):
        if self.config['filter_inter_by_user_or_item'] is not True:
            return
        keep = pd.Series(True, index=self.inter_feat.index)
        if self.user_feat is not None:
            keep &= self.inter_feat[self.uid_field].isin(self.user_feat[self.uid_field].values)
        if self.item_feat is not None:
            keep &= self.inter_feat[self.iid_field].isin(self.item_feat[self.iid_field].values)
        self.inter_feat.drop(self.inter_feat.index[~keep], inplace=True)

    def _illegal_ids(self, field, feat, inter_num, max_num, min_num):
        max_num = max_num or np.inf
        min_num = min_num or -1
        ids = {i for i in inter_num if inter_num[i] < min_num or inter_num[i] > max_num}
        if feat is not None:
            for i in feat[field].values:
                if inter_num[i] < min_num:
                    ids.add(i)
        return ids

    def _filter_by_inter_num(self):
        if self.uid_field is None or self.iid_field is None:
            return
        mxu, mnu = self.config['max_user_inter_num'], self.config['min_user_inter_num']
        mxi, mni = self.config['max_item_inter_num'], self.config['min_item_inter_num']
        # a bound of None / 0 on both sides can drop nothing (_illegal_ids: counts are
        # >= 0 > -1 and < inf): skip the counting; else hash counts in C (value_counts)
        # instead of a Python Counter over every interaction
        uc = Counter() if mxu is None and not mnu else _counts(self.inter_feat[self.uid_field])
        ic = Counter() if mxi is None and not mni else _counts(self.inter_feat[self.iid_field])
        while True:
            bu = self._illegal_ids(self.uid_field, self.user_feat, uc, mxu, mnu)
            bi = self._illegal_ids(self.iid_field, self.item_feat, ic, mxi, mni)
            if not bu and not bi:
                break
            if self.user_feat is not None:
                d = self.user_feat[self.uid_field].isin(bu)
                self.user_feat.drop(self.user_feat.index[d], inplace=True)
            if self.item_feat is not None:
                d = self.item_feat[self.iid_field].isin(bi)
                self.item_feat.drop(self.item_feat.index[d], inplace=True)
            ui, ii = self.inter_feat[self.uid_field], self.inter_feat[self.iid_field]
            dropped = ui.isin(bu) | ii.isin(bi)
            uc -= _counts(ui[dropped])
            ic -= _counts(ii[dropped])
            self.inter_feat.drop(self.inter_feat.index[dropped], inplace=True)

    def _reset_index(self):
        for fname in self.feat_name_list:
            feat = getattr(self, fname)
            if feat.empty:
                raise ValueError('Some feat is empty, please check the filtering settings.')
            feat.reset_index(drop=True, inplace=True)

    # ------------------------------------------------------------------ remap
    def _get_fields_in_same_space(self):
        fss = self.config['fields_in_same_space'] or []
        fss = [set(s) for s in fss]
        additional = []
        token_like = {FeatureType.TOKEN, FeatureType.TOKEN_SEQ}
        for field in self.field2source:
            if self.field2type[field] not in token_like:
                continue
            if any(field in s for s in fss):
                continue
            additional.append({field})
        return fss + additional

    def _get_remap_list(self, field_set):
        remap = []
        field_set = set(field_set)
        for field, feat in [(self.uid_field, self.user_feat), (self.iid_field, self.item_feat)]:
            if field in field_set:
                field_set.remove(field)
                remap.append((self.inter_feat, field, FeatureType.TOKEN))
                if feat is not None:
                    remap.append((feat, field, FeatureType.TOKEN))
        for field in field_set:
            src = self.field2source[field]
            src = src.value if isinstance(src, FeatureSource) else src
            if src in ('user_id', 'item_id'):
                src = src.split('_')[0]
            feat = getattr(self, f'{src}_feat')
            remap.append((feat, field, self.field2type[field]))
        return remap

    def _remap_ID_all(self):
        for field_set in self._get_fields_in_same_space():
            self._remap(self._get_remap_list(field_set))

    def _remap(self, remap_list):
        tokens = []
        for feat, field, ftype in remap_list:
            if ftype == FeatureType.TOKEN:
                tokens.append(feat[field].values)
            else:
                vals = feat[field].values
                tokens.append(np.concatenate(list(vals)) if len(vals) else np.array([]))
        if not tokens:
            return
        split_point = np.cumsum([len(t) for t in tokens])[:-1]
        new_ids, mp = _factorize(tokens)
        new_ids_list = np.split(new_ids + 1, split_point)
        mp = np.array(['[PAD]'] + list(mp))
        token_id = {t: i for i, t in enumerate(mp)}
        for (feat, field, ftype), ids in zip(remap_list, new_ids_list):
            if field not in self.field2id_token:
                self.field2id_token[field] = mp
                self.field2token_id[field] = token_id
            if ftype == FeatureType.TOKEN:
                feat[field] = ids
            else:
                sp = np.cumsum([len(x) for x in feat[field].values])[:-1]
                feat[field] = np.split(ids, sp)

    # ------------------------------------------------------------------ prep
    def _user_item_feat_preparation(self):
        if self.user_feat is not None:
            base = pd.DataFrame({self.uid_field: np.arange(self.user_num)})
            self.user_feat = pd.merge(base, self.user_feat, on=self.uid_field, how='left')
        if self.item_feat is not None:
            base = pd.DataFrame({self.iid_field: np.arange(self.item_num)})
            self.item_feat = pd.merge(base, self.item_feat, on=self.iid_field, how='left')

    def _fill_nan(self):
        for fname in self.feat_name_list:
            feat = getattr(self, fname)
            for field in feat:
                ftype = self.field2type[field]
                if ftype == FeatureType.TOKEN:
                    feat[field] = feat[field].fillna(value=0)
                elif ftype == FeatureType.FLOAT:
                    feat[field] = feat[field].fillna(value=feat[field].mean())
                else:
                    dt = np.int64 if ftype == FeatureType.TOKEN_SEQ else np.float64
                    feat[field] = feat[field].apply(
                        lambda x: np.array([], dtype=dt) if isinstance(x, float) else x)

    def _set_label_by_threshold(self):
        threshold = self.config['threshold']
        if threshold is None:
            return
        if len(threshold) != 1:
            raise ValueError('Threshold length should be 1.')
        self.set_field_property(self.label_field, FeatureType.FLOAT, FeatureSource.INTERACTION, 1)
        for field, value in threshold.items():
            if field in self.inter_feat:
                self.inter_feat[self.label_field] = (self.inter_feat[field] >= value).astype(int)
            else:
                raise ValueError(f'Field [{field}] not in inter_feat.')
            if field != self.label_field:
                self._del_col(self.inter_feat, field)

    def set_field_property(self, field, ftype, source, seqlen):
        self.field2type[field] = ftype
        self.field2source[field] = source
        self.field2seqlen[field] = seqlen

    def copy_field_property(self, dest_field, source_field):
        self.field2type[dest_field] = self.field2type[source_field]
        self.field2source[dest_field] = self.field2source[source_field]
        self.field2seqlen[dest_field] = self.field2seqlen[source_field]

    def to_device(self, device):
        """Move inter/user/item features to `device` (the train loaders keep
        their columns resident in HBM; slicing then stays on the GPU)."""
        for fname in self.feat_name_list:
            feat = getattr(self, fname)
            if isinstance(feat, Interaction):
                setattr(self, fname, feat.to(device))
        return self

    def _del_col(self, feat, field):
        if isinstance(feat, Interaction):
            feat.drop(column=field)
        else:
            feat.drop(columns=field, inplace=True)
        for d in [self.field2id_token, self.field2token_id, self.field2seqlen, self.field2source,
                  self.field2type]:
            d.pop(field, None)

    @property
    def float_like_fields(self):
        return [f for f, t in self.field2type.items()
                if t in {FeatureType.FLOAT, FeatureType.FLOAT_SEQ}]

    def _normalize(self):
        if self.config['normalize_field'] is not None and self.config['normalize_all'] is True:
            raise ValueError("Normalize_field and normalize_all can't be set at the same time.")
        if self.config['normalize_field']:
            fields = self.config['normalize_field']
        elif self.config['normalize_all']:
            fields = self.float_like_fields
        else:
            return
        for fname in self.feat_name_list:
            feat = getattr(self, fname)
            for field in list(feat.columns):
                if field not in fields:
                    continue
                ftype = self.field2type[field]
                if ftype == FeatureType.FLOAT:
                    lst = feat[field].values
                    mx, mn = max(lst), min(lst)
                    feat[field] = 1.0 if mx == mn else (lst - mn) / (mx - mn)
                elif ftype == FeatureType.FLOAT_SEQ:
                    sp = np.cumsum([len(x) for x in feat[field].values])[:-1]
                    lst = np.concatenate(list(feat[field].values))
                    mx, mn = max(lst), min(lst)
                    lst = np.ones_like(lst) if mx == mn else (lst - mn) / (mx - mn)
                    feat[field] = np.split(lst, sp)

    # ------------------------------------------------------------------ API
    def token2id(self, field, tokens):
        """External token(s) -> internal id(s) (reference dataset.py:1040-1058):
        ValueError for an unknown token, TypeError for another input type."""
        if isinstance(tokens, str):
            if tokens in self.field2token_id[field]:
                return self.field2token_id[field][tokens]
            raise ValueError(f'token [{tokens}] is not existed in {field}')
        if isinstance(tokens, (list, np.ndarray)):
            return np.array([self.token2id(field, t) for t in tokens])
        raise TypeError(f'The type of tokens [{tokens}] is not supported')

    def id2token(self, field, ids):
        """Internal id(s) -> external token(s) (reference dataset.py:1082-1098)."""
        try:
            return self.field2id_token[field][ids]
        except IndexError:
            if isinstance(ids, list):
                raise ValueError(f'[{ids}] is not a one-dimensional list.')
            raise ValueError(f'[{ids}] is not a valid ids.')

    def num(self, field):
        if field not in self.field2type:
            raise ValueError(f'Field [{field}] not defined in dataset.')
        if self.field2type[field] not in {FeatureType.TOKEN, FeatureType.TOKEN_SEQ}:
            return self.field2seqlen[field]
        return len(self.field2id_token[field])

    @property
    def user_num(self):
        return self.num(self.uid_field)

    @property
    def item_num(self):
        return self.num(self.iid_field)

    @property
    def inter_num(self):
        return len(self.inter_feat)

    def fields(self, ftype=None, source=None):
        ftype = set(ftype) if ftype is not None else set(FeatureType)
        source = set(source) if source is not None else set(FeatureSource)
        return [f for f in self.field2type
                if self.field2type[f] in ftype and self.field2source[f] in source]

    @property
    def token_like_fields(self):
        return self.fields(ftype=[FeatureType.TOKEN, FeatureType.TOKEN_SEQ])

    def _dataframe_to_interaction(self, data):
        new = {}
        for k in data:
            value = data[k].values
            ftype = self.field2type[k]
            if ftype == FeatureType.TOKEN:
                new[k] = torch.LongTensor(np.asarray(value, dtype=np.int64))
            elif ftype == FeatureType.FLOAT:
                new[k] = torch.FloatTensor(np.asarray(value, dtype=np.float64))
            elif ftype == FeatureType.TOKEN_SEQ:
                seqs = [torch.LongTensor(np.asarray(d[:self.field2seqlen[k]], dtype=np.int64))
                        for d in value]
                new[k] = torch.nn.utils.rnn.pad_sequence(seqs, batch_first=True)
            else:
                seqs = [torch.FloatTensor(np.asarray(d[:self.field2seqlen[k]], dtype=np.float64))
                        for d in value]
                new[k] = torch.nn.utils.rnn.pad_sequence(seqs, batch_first=True)
        return Interaction(new)

    def _change_feat_format(self):
        for fname in self.feat_name_list:
            feat = getattr(self, fname)
            if isinstance(feat, pd.DataFrame):
                setattr(self, fname, self._dataframe_to_interaction(feat))

    def _drop_unused_col(self):
        unused = self.config['unused_col']
        if unused is None:
            return
        for fname, fields in unused.items():
            feat = getattr(self, fname + '_feat')
            for field in fields:
                if field in feat:
                    self._del_col(feat, field)

    def _calcu_split_ids(self, tot, ratios):
        """dataset.py:1258-1279 (first part takes the remainder)."""
        cnt = [int(ratios[i] * tot) for i in range(len(ratios))]
        cnt[0] = tot - sum(cnt[1:])
        for i in range(1, len(ratios)):
            if cnt[0] <= 1:
                break
            if 0 < ratios[-i] * tot < 1:
                cnt[-i] += 1
                cnt[0] -= 1
        return list(np.cumsum(cnt)[:-1])

    @staticmethod
    def _grouped_index(group_by_list):
        """Row indices per group, groups in first-appearance order (dataset.py:1249-1256)."""
        keys = np.asarray(group_by_list)
        if len(keys) == 0:
            return []
        order = _stable_order(keys)
        sk = keys[order]
        starts = np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]])
        ends = np.r_[starts[1:], len(sk)]
        first = order[starts]
        groups = [order[s:e] for s, e in zip(starts, ends)]
        return [groups[i] for i in np.argsort(first, kind='stable')]

    def split_by_ratio(self, ratios, group_by=None):
        tot_ratio = sum(ratios)
        ratios = [r / tot_ratio for r in ratios]
        if group_by is None:
            tot = len(self)
            split_ids = self._calcu_split_ids(tot, ratios)
            next_index = [np.arange(s, e) for s, e in zip([0] + split_ids, split_ids + [tot])]
        else:
            next_index = _grouped_ratio_split(self.inter_feat[group_by].numpy(), ratios)
        self._drop_unused_col()
        return [self.copy(self.inter_feat[torch.as_tensor(np.asarray(ix, dtype=np.int64))])
                for ix in next_index]

    def leave_one_out(self, group_by, leave_one_num=1):
        if group_by is None:
            raise ValueError('leave one out strategy require a group field')
        nxt = _grouped_leave_one_out(self.inter_feat[group_by].numpy(), leave_one_num)
        self._drop_unused_col()
        return [self.copy(self.inter_feat[torch.as_tensor(np.asarray(ix, dtype=np.int64))])
                for ix in nxt]

    def shuffle(self):
        return self.inter_feat.shuffle()

    def sort(self, by, ascending=True):
        self.inter_feat.sort(by=by, ascending=ascending)

    def build(self, eval_setting):
        self._change_feat_format()
        if self.benchmark_filename_list is not None:
            cs = list(np.cumsum(self.file_size_list))
            return [self.copy(self.inter_feat[s:e]) for s, e in zip([0] + cs[:-1], cs)]
        oa = eval_setting.ordering_args
        if oa['strategy'] == 'shuffle':
            self.shuffle()
        elif oa['strategy'] == 'by':
            self.sort(by=oa['field'], ascending=oa['ascending'])
        sa = eval_setting.split_args
        if sa['strategy'] == 'by_ratio':
            return self.split_by_ratio(sa['ratios'], group_by=eval_setting.group_field)
        if sa['strategy'] == 'by_value':
            raise NotImplementedError()
        if sa['strategy'] == 'loo':
            return self.leave_one_out(group_by=eval_setting.group_field,
                                      leave_one_num=sa['leave_one_num'])
        return self

    def copy(self, new_inter_feat):
        nxt = copy.copy(self)
        nxt.inter_feat = new_inter_feat
        return nxt

    def join(self, df):
        if self.user_feat is not None and self.uid_field in df:
            df.update(self.user_feat[df[self.uid_field]])
        if self.item_feat is not None and self.iid_field in df:
            df.update(self.item_feat[df[self.iid_field]])
        return df

    def __getitem__(self, index, join=True):
        df = self.inter_feat[index]
        return self.join(df) if join else df

    def __len__(self):
        return len(self.inter_feat)

    def __str__(self):
        return (f'{self.dataset_name}\nThe number of users: {self.user_num}\n'
                f'The number of items: {self.item_num}\nThe number of inters: {self.inter_num}\n'
                f'Remain Fields: {list(self.field2type)}')

    __repr__ = __str__

    def get_item_feature(self):
        if self.item_feat is None:
            return Interaction({self.iid_field: torch.arange(self.item_num)})
        return self.item_feat

    def inter_matrix(self, form='coo', value_field=None):
        """User x item sparse matrix of this split (dataset.py:1538-1557)."""
        import scipy.sparse as sp
        src = self.inter_feat[self.uid_field].cpu().numpy()
        tgt = self.inter_feat[self.iid_field].cpu().numpy()
        data = np.ones(len(self.inter_feat)) if value_field is None else \
            self.inter_feat[value_field].cpu().numpy()
        mat = sp.coo_matrix((data, (src, tgt)), shape=(self.user_num, self.item_num))
        if form == 'coo':
            return mat
        if form == 'csr':
            return mat.tocsr()
        raise NotImplementedError(f'sparse matrix format [{form}] has not been implemented.')
