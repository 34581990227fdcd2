"""Default configuration values, restated as Python data from the reference's
property files (recbole/properties/overall.yaml, dataset/sample.yaml,
dataset/ml-100k.yaml, model/{BPR,LightGCN,SASRec,DeepFM}.yaml,
quick_start_config/{sequential,context-aware}.yaml)."""
from recbole_amd.utils.enum_type import ModelType

OVERALL = dict(
    # general
    gpu_id=0, use_gpu=True, seed=2020, state='INFO', reproducibility=True,
    data_path='dataset/', checkpoint_dir='saved', show_progress=True,
    # training
    epochs=300, train_batch_size=2048, learner='adam', learning_rate=0.001,
    training_neg_sample_num=1, training_neg_sample_distribution='uniform', eval_step=1,
    stopping_step=10, clip_grad_norm=None, weight_decay=0.0, draw_loss_pic=False,
    # evaluation
    eval_setting='RO_RS,full', group_by_user=True, split_ratio=[0.8, 0.1, 0.1],
    leave_one_num=2, real_time_process=False,
    metrics=['Recall', 'MRR', 'NDCG', 'Hit', 'Precision'], topk=[10],
    valid_metric='MRR@10', eval_batch_size=4096, loss_decimal_place=4,
    metric_decimal_place=4,
    # MI355X build extensions
    n_gpus=None, fused_train=True, fused_eval=True, train_graph=True, profile=False,
    adam_mode='deferred', shard_tables=True,
    neg_sampling_alias=False,   # alias-table fast mode (NON-PARITY, sampler.enable_alias)
)

SAMPLE = dict(
    field_separator='\t', seq_separator=' ',
    USER_ID_FIELD='user_id', ITEM_ID_FIELD='item_id', RATING_FIELD='rating',
    TIME_FIELD='timestamp', seq_len=None, LABEL_FIELD='label', threshold=None,
    NEG_PREFIX='neg_', load_col={'inter': ['user_id', 'item_id']}, unload_col=None,
    unused_col=None, additional_feat_suffix=None,
    rm_dup_inter=None, lowest_val=None, highest_val=None, equal_val=None, not_equal_val=None,
    filter_inter_by_user_or_item=True, max_user_inter_num=None, min_user_inter_num=0,
    max_item_inter_num=None, min_item_inter_num=0,
    fields_in_same_space=None, preload_weight=None, normalize_field=None, normalize_all=None,
    ITEM_LIST_LENGTH_FIELD='item_length', LIST_SUFFIX='_list', MAX_ITEM_LIST_LENGTH=50,
    POSITION_FIELD='position_id',
    HEAD_ENTITY_ID_FIELD='head_id', TAIL_ENTITY_ID_FIELD='tail_id',
    RELATION_ID_FIELD='relation_id', ENTITY_ID_FIELD='entity_id',
    SOURCE_ID_FIELD='source_id', TARGET_ID_FIELD='target_id',
    benchmark_filename=None,
    # keys the reference reads with .get-like semantics
    group_field=None, ordering_args=None, split_args=None, neg_sample_args=None,
    train_use_bothway_sampler=None, eval_use_bothway_sampler=None,
)

DATASET_DEFAULTS = {
    'ml-100k': dict(
        load_col={'inter': ['user_id', 'item_id', 'rating', 'timestamp'],
                  'item': ['item_id', 'movie_title', 'class', 'tags']},
        min_user_inter_num=None, min_item_inter_num=None, normalize_all=True,
    ),
}

MODEL_DEFAULTS = {
    'BPR': dict(embedding_size=64),
    'LightGCN': dict(embedding_size=64, n_layers=2, reg_weight=1e-05),
    'SASRec': dict(n_layers=2, n_heads=2, hidden_size=64, inner_size=256,
                   hidden_dropout_prob=0.5, attn_dropout_prob=0.5, hidden_act='gelu',
                   layer_norm_eps=1e-12, initializer_range=0.02, loss_type='CE'),
    'DeepFM': dict(embedding_size=10, mlp_hidden_size=[128, 128, 128], dropout_prob=0.2),
}

# quick_start_config/context-aware_ml-100k.yaml, applied after the type preset
TYPE_DATASET_PRESETS = {
    (ModelType.CONTEXT, 'ml-100k'): dict(
        threshold={'rating': 4},
        load_col={'inter': ['user_id', 'item_id', 'rating', 'timestamp'],
                  'user': ['user_id', 'age', 'gender', 'occupation'],
                  'item': ['item_id', 'release_year', 'class']}),
}

TYPE_PRESETS = {
    ModelType.SEQUENTIAL: dict(eval_setting='TO_LS,full'),
    ModelType.CONTEXT: dict(eval_setting='RO_RS', group_by_user=False, training_neg_sample_num=0,
                            metrics=['AUC', 'LogLoss'], valid_metric='AUC'),
}
