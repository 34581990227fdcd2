"""Dataset classes, laid out as the reference's package (recbole/data/dataset/__init__.py:1-2):
`recbole.data.dataset.Dataset`, `recbole.data.dataset.SequentialDataset` and the
module paths `recbole.data.dataset.dataset` / `.sequential_dataset` resolve here."""
from recbole_amd.data.dataset.dataset import Dataset
from recbole_amd.data.dataset.sequential_dataset import SequentialDataset

__all__ = ['Dataset', 'SequentialDataset']
