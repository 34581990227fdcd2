"""Registry of dataset attributes every loader proxies (the reference's DLFriendlyAPI,
data/utils.py:352-393: `@dlapi.set()` on a Dataset method makes `loader.<name>` the
dataset's). Seeded with the names the models of this build read through their train
loader (`Model(config, train_data)`: num, fields, field2type, inter_matrix, ...)."""


class DLFriendlyAPI(object):

    def __init__(self, names=()):
        self.dataloader_apis = set(names)

    def __iter__(self):
        return iter(sorted(self.dataloader_apis))

    def set(self):
        """Decorator: register a Dataset method / property name."""
        def register(f):
            self.dataloader_apis.add(f.__name__)
            return f
        return register


# the reference's decorated Dataset methods (num ... get_preload_weight) plus the field
# tables and id fields its models read from the loader
dlapi = DLFriendlyAPI(('num', 'fields', 'token2id', 'token2id_exists', 'id2token', 'user_num',
                       'item_num', 'join', 'get_user_feature', 'get_item_feature',
                       'inter_matrix', 'history_item_matrix', 'history_user_matrix',
                       'get_preload_weight', 'field2type', 'field2source', 'field2id_token',
                       'field2token_id', 'field2seqlen', 'uid_field', 'iid_field'))
