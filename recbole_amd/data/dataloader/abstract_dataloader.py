"""Iterator protocol shared by all loaders (mirror of
recbole/data/dataloader/abstract_dataloader.py:21-133)."""
import math
from logging import getLogger

from recbole_amd.data.dlapi import dlapi
from recbole_amd.utils import InputType


class AbstractDataLoader(object):
    dl_type = None

    def __init__(self, config, dataset, batch_size=1, dl_format=InputType.POINTWISE, shuffle=False):
        self.config = config
        self.logger = getLogger()
        self.dataset = dataset
        self.batch_size = batch_size
        self.step = batch_size
        self.dl_format = dl_format
        self.shuffle = shuffle
        self.pr = 0
        self.real_time = config['real_time_process']
        if self.real_time is None:
            self.real_time = True
        # dataset APIs proxied to the loader (data/utils.py:352-393 dlapi); the loader's
        # own methods (get_user_feature, ...) take precedence
        for attr in dlapi:
            if hasattr(self.dataset, attr) and not hasattr(type(self), attr):
                setattr(self, attr, getattr(self.dataset, attr))
        self.setup()
        if not self.real_time:
            self.data_preprocess()

    def setup(self):
        pass

    def data_preprocess(self):
        pass

    def __len__(self):
        return math.ceil(self.pr_end / self.step)

    def __iter__(self):
        if self.shuffle:
            self._shuffle()
        return self

    def __next__(self):
        if self.pr >= self.pr_end:
            self.pr = 0
            raise StopIteration()
        return self._next_batch_data()

    @property
    def pr_end(self):
        raise NotImplementedError('Method [pr_end] should be implemented')

    def _shuffle(self):
        raise NotImplementedError('Method [shuffle] should be implemented.')

    def _next_batch_data(self):
        raise NotImplementedError('Method [next_batch_data] should be implemented.')

    def set_batch_size(self, batch_size):
        if self.pr != 0:
            raise PermissionError("Cannot change dataloader's batch_size while iteration")
        if self.batch_size != batch_size:
            self.batch_size = batch_size
            self.logger.warning(f'Batch size is changed to {batch_size}.')

    def upgrade_batch_size(self, batch_size):
        if self.batch_size < batch_size:
            self.set_batch_size(batch_size)

    def get_user_feature(self):
        return self.dataset.user_feat

    def get_item_feature(self):
        return self.dataset.get_item_feature()
