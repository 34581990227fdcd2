"""Evaluation presets (mirror of recbole/config/eval_setting.py:18-391):
ordering (RO = shuffle, TO = by timestamp), splitting (RS = by ratio,
LS = leave-one-out), grouped by user, and the negative-sampling presets
full / uniN / popN."""
import re

from recbole_amd.utils import set_color


class EvalSetting(object):

    def __init__(self, config):
        self.config = config
        self.group_field = None
        self.ordering_args = None
        self.split_args = None
        self.neg_sample_args = {'strategy': 'none'}
        self.es_str = [s.strip() for s in config['eval_setting'].split(',')]
        self.set_ordering_and_splitting(self.es_str[0])
        if len(self.es_str) > 1:
            self._set_neg_preset(self.es_str[1])
        for args in ['group_field', 'ordering_args', 'split_args', 'neg_sample_args']:
            if config[args] is not None:
                setattr(self, args, config[args])

    def _set_neg_preset(self, s):
        if s == 'full':
            self.neg_sample_args = {'strategy': 'full', 'distribution': 'uniform'}
            return
        m = re.fullmatch(r'(uni|pop)(\d+)', s)
        if m is None:
            raise ValueError('Incorrect setting of negative sampling.')
        dist = 'uniform' if m.group(1) == 'uni' else 'popularity'
        self.neg_sample_args = {'strategy': 'by', 'by': int(m.group(2)), 'distribution': dist}

    def set_ordering_and_splitting(self, es_str):
        args = es_str.split('_')
        if len(args) != 2:
            raise ValueError(f'`{es_str}` is invalid eval_setting.')
        ordering, split = args
        if self.config['group_by_user']:
            self.group_field = self.config['USER_ID_FIELD']
        if ordering == 'RO':
            self.ordering_args = {'strategy': 'shuffle'}
        elif ordering == 'TO':
            self.ordering_args = {'strategy': 'by', 'field': self.config['TIME_FIELD'],
                                  'ascending': True}
        else:
            raise NotImplementedError(f'Ordering args `{ordering}` is not implemented.')
        if split == 'RS':
            ratios = self.config['split_ratio']
            if ratios is None:
                raise ValueError('`ratios` should be set if `RS` is set.')
            self.split_args = {'strategy': 'by_ratio', 'ratios': ratios}
        elif split == 'LS':
            n = self.config['leave_one_num']
            if n is None:
                raise ValueError('`leave_one_num` should be set if `LS` is set.')
            self.split_args = {'strategy': 'loo', 'leave_one_num': n}
        else:
            raise NotImplementedError(f'Split args `{split}` is not implemented.')

    def __str__(self):
        info = [set_color('Evaluation Setting:', 'pink'),
                f'Group by {self.group_field}' if self.group_field else 'No Grouping',
                f'Ordering: {self.ordering_args}', f'Splitting: {self.split_args}',
                f'Negative Sampling: {self.neg_sample_args}']
        return '\n\t'.join(info)

    __repr__ = __str__
