"""Context-aware host logic on the CPU: the dataset pipeline for token / float /
token_seq fields, DeepFM's module tree (state_dict keys and shapes identical to
the oracle's restatement of the reference tree, so checkpoints interoperate) and
the K8 field layout (concat order token | token_seq | float, offsets)."""
import numpy as np

from oracle import cpu_ref
from tests.ctx_data import write_ctx_dataset


def test_deepfm_layout_and_state_dict(tmp_path):
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.utils import get_model, init_seed
    root = write_ctx_dataset(str(tmp_path))
    config = Config(config_dict={'model': 'DeepFM', 'dataset': 'ctx', 'data_path': root,
                                 'embedding_size': 16, 'load_col': None, 'use_gpu': False})
    init_seed(config['seed'], config['reproducibility'])
    ds = create_dataset(config)
    train, valid, test = data_preparation(config, ds)
    assert len(train.dataset) + len(valid.dataset) + len(test.dataset) == 3000
    m = get_model('DeepFM')(config, train)
    lay = m.field_layout
    assert lay.token_names == ['user_id', 'item_id', 'C0', 'C1', 'C2', 'C3']
    assert lay.seq_names == ['tags'] and lay.float_names == ['I0', 'I1', 'I2']
    assert lay.token_offsets == list(np.r_[0, np.cumsum(m.token_field_dims)[:-1]])
    ref = cpu_ref.DeepFMCPU(m.token_field_names, m.token_field_dims, m.token_seq_field_names,
                            m.token_seq_field_dims, m.float_field_names, 16,
                            m.mlp_hidden_size, 0.0)
    a = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    b = {k: tuple(v.shape) for k, v in ref.state_dict().items()}
    assert a == b
    assert m.mlp_layers.mlp_layers[1].in_features == 16 * 10
    batch = next(iter(train))
    assert batch['tags'].dim() == 2 and batch['I0'].dtype.is_floating_point
