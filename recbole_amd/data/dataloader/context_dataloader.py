"""Context-aware loaders (mirror of recbole/data/dataloader/context_dataloader.py:19-40).

In the reference these three classes subclass the General* loaders without changing
anything; they exist so that `get_data_loader` can resolve `Context` + strategy by
name for context-aware models (DeepFM). The same holds here: a context model's batch
is the General loader's batch (token / float columns joined on the device)."""
from recbole_amd.data.dataloader.general_dataloader import (GeneralDataLoader,
                                                            GeneralFullDataLoader,
                                                            GeneralNegSampleDataLoader)


class ContextDataLoader(GeneralDataLoader):
    """GeneralDataLoader under the name `get_data_loader` builds for ModelType.CONTEXT."""


class ContextNegSampleDataLoader(GeneralNegSampleDataLoader):
    """GeneralNegSampleDataLoader for ModelType.CONTEXT."""


class ContextFullDataLoader(GeneralFullDataLoader):
    """GeneralFullDataLoader for ModelType.CONTEXT."""
