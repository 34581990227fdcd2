"""Trainer (mirror of recbole/trainer/trainer.py:38-452).

Same constructor, fit/evaluate signatures, logging lines, early stopping and
checkpoint dict as the reference. Two execution paths:

* fused (default when applicable: model exposes fused_embedding_tables(),
  learner 'adam', no clip_grad_norm, pairwise train loader on the GPU):
  recbole_amd/trainer/fused.py runs the whole step as hand-written kernels and
  keeps per-batch losses on the device until the end of the epoch;
* generic: the reference's loop (to(device) -> zero_grad -> calculate_loss ->
  item -> NaN check -> backward -> clip -> step), with the model's own
  kernels inside calculate_loss and FusedAdam (or torch's learners) as step.

Evaluation of a FULL loader uses the fused K6 scorer when the model provides
fused_user_vectors()/fused_item_table(); otherwise the reference's
full_sort_predict + mask + swap + TopKEvaluator.collect sequence.

Documented difference: the NaN check of the fused path runs once per epoch
(the reference checks every batch, trainer.py:169, at the cost of a host sync
per batch); a NaN still raises ValueError('Training loss is nan').
"""
from __future__ import annotations

import os
from logging import getLogger
from time import time

import numpy as np
import torch
import torch.optim as optim
from torch.nn.utils.clip_grad import clip_grad_norm_

from recbole_amd.data.dataloader.general_dataloader import GeneralNegSampleDataLoader
from recbole_amd.evaluator import ProxyEvaluator
from recbole_amd.data.dataloader.sequential_dataloader import SequentialNegSampleDataLoader
from recbole_amd.sampler import RepeatableSampler
from recbole_amd.trainer.fused import (FusedBPRTrainStep, ShardedBPRTrainStep,
                                       fused_full_sort_eval,
                                       fused_general_sampled_eval, fused_seq_full_sort_eval,
                                       fused_seq_sampled_eval)
from recbole_amd.trainer.dist import DataParallelStep, active_group
from recbole_amd.trainer.optim import FusedAdam
from recbole_amd.utils import (DataLoaderType, InputType, calculate_valid_score, dict2str,
                               early_stopping, ensure_dir, get_local_time, set_color)


class AbstractTrainer(object):

    def __init__(self, config, model):
        self.config = config
        self.model = model

    def fit(self, train_data):
        raise NotImplementedError('Method [next] should be implemented.')

    def evaluate(self, eval_data):
        raise NotImplementedError('Method [next] should be implemented.')


class Trainer(AbstractTrainer):

    def __init__(self, config, model):
        super().__init__(config, model)
        self.logger = getLogger()
        self.learner = config['learner']
        self.learning_rate = config['learning_rate']
        self.epochs = config['epochs']
        self.eval_step = min(config['eval_step'], self.epochs)
        self.stopping_step = config['stopping_step']
        self.clip_grad_norm = config['clip_grad_norm']
        self.valid_metric = config['valid_metric'].lower()
        self.valid_metric_bigger = config['valid_metric_bigger']
        self.test_batch_size = config['eval_batch_size']
        self.device = config['device']
        self.checkpoint_dir = config['checkpoint_dir']
        ensure_dir(self.checkpoint_dir)
        self.saved_model_file = os.path.join(self.checkpoint_dir,
                                             f"{config['model']}-{get_local_time()}.pth")
        self.weight_decay = config['weight_decay']
        self.draw_loss_pic = config['draw_loss_pic']
        self.start_epoch = 0
        self.cur_step = 0
        self.best_valid_score = -np.inf if self.valid_metric_bigger else np.inf
        self.best_valid_result = None
        self.train_loss_dict = dict()
        self.optimizer = self._build_optimizer(self.model.parameters())
        self._dp = None
        group = active_group(config)
        if group is not None:
            self._dp = DataParallelStep(group)
        if (isinstance(self.optimizer, FusedAdam) and config['adam_mode'] != 'streamed'
                and hasattr(self.model, 'deferred_tables')):
            # sparsely read embedding tables on the deferred K5 schedule (optim.py)
            self.optimizer.enable_deferred(self.model.deferred_tables())
            if self._dp is not None and config['shard_tables'] is not False:
                # data parallel: the deferred tables row-sharded over the ranks (optim.py)
                self.optimizer.shard_deferred(self._dp.group)
            # any state_dict() of the model sees complete rows
            self.model.register_state_dict_pre_hook(lambda *a, **k: self.optimizer.flush())
        self.eval_type = config['eval_type']
        self.evaluator = ProxyEvaluator(config)
        self.item_tensor = None
        self.tot_item_num = None
        self._fused_step = None

    def _build_optimizer(self, params):
        """trainer.py:109-130; 'adam' runs on the K5 kernel (FusedAdam)."""
        name = self.learner.lower()
        if name == 'adam':
            return FusedAdam(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == 'sgd':
            return optim.SGD(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == 'adagrad':
            return optim.Adagrad(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == 'rmsprop':
            return optim.RMSprop(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == 'sparse_adam':
            if self.weight_decay > 0:
                self.logger.warning('Sparse Adam cannot argument received argument [{weight_decay}]')
            return optim.SparseAdam(params, lr=self.learning_rate)
        self.logger.warning('Received unrecognized optimizer, set default Adam optimizer')
        return FusedAdam(params, lr=self.learning_rate)

    # ------------------------------------------------------------------ training
    def _fused_applicable(self, train_data):
        if not self.config['fused_train'] or self.clip_grad_norm:
            return False
        if not isinstance(self.optimizer, FusedAdam):
            return False
        if not hasattr(self.model, 'fused_embedding_tables'):
            return False
        if not isinstance(train_data, GeneralNegSampleDataLoader):
            return False
        if train_data.dl_format != InputType.PAIRWISE or train_data.user_inter_in_one_batch:
            return False
        tables = {id(p) for p, _ in self.model.fused_embedding_tables()}
        params = [p for p in self.model.parameters() if p.requires_grad]
        if {id(p) for p in params} != tables:
            return False
        return all(p.is_cuda for p in params)

    def _train_epoch(self, train_data, epoch_idx, loss_func=None, show_progress=False):
        self.model.train()
        if loss_func is None and self._fused_applicable(train_data):
            if self._fused_step is None or self._fused_step.data is not train_data:
                mode = self.config['adam_mode'] or 'deferred'
                # data parallel: row-sharded tables unless
                # shard_tables: False asks for replicas
                cls = (ShardedBPRTrainStep if self._dp is not None and mode == 'deferred'
                       and self.config['shard_tables'] is not False else FusedBPRTrainStep)
                # fused_step (K35, one launch per step): None = where it applies
                kw = {} if cls is ShardedBPRTrainStep else {'fused_step': self.config['fused_step']}
                self._fused_step = cls(
                    self.model, self.optimizer, train_data,
                    use_graph=self.config['train_graph'] is not False, adam_mode=mode,
                    dist=self._dp.group if self._dp is not None else None, **kw)
            losses = self._fused_step.run_epoch()
            total = None
            for v in losses:
                total = v if total is None else total + v
                if np.isnan(v):
                    raise ValueError('Training loss is nan')
            return total
        if loss_func is None and self._graph_step_applicable():
            return self._train_epoch_graphed(train_data)
        loss_func = loss_func or self.model.calculate_loss
        total_loss = None
        dp = self._dp
        for batch_idx, interaction in enumerate(train_data):
            interaction = interaction.to(self.device)
            shard = False
            if dp is not None:                 # data parallel: this rank's slice (dist.py)
                interaction, shard = dp.local_slice(interaction)
            self.optimizer.zero_grad()
            losses = loss_func(interaction)
            # reported values: the global-batch mean when sharded
            shown = (lambda x: dp.global_loss(x).item()) if shard else (lambda x: x.item())
            if isinstance(losses, tuple):
                loss = sum(losses)
                lt = tuple(shown(x) for x in losses)
                total_loss = lt if total_loss is None else tuple(map(sum, zip(total_loss, lt)))
            else:
                loss = losses
                v = shown(losses)
                total_loss = v if total_loss is None else total_loss + v
            self._check_nan(loss)
            (loss * dp.loss_scale() if shard else loss).backward()
            if shard:
                dp.exchange(self.model, self.optimizer)
            if self.clip_grad_norm:
                clip_grad_norm_(self.model.parameters(), **self.clip_grad_norm)
            self.optimizer.step()
        self._sync_params()
        return total_loss

    def _graph_step_applicable(self):
        """The captured generic step (trainer/graph_step.py): FusedAdam, one process,
        no gradient clipping, and a model whose training step is capture-safe."""
        return (self.config['train_graph'] is not False and isinstance(self.optimizer, FusedAdam)
                and self._dp is None and not self.clip_grad_norm
                and getattr(self.model, 'graph_step_safe', False)
                and next(self.model.parameters()).is_cuda)

    def _train_epoch_graphed(self, train_data):
        """_train_epoch with each full batch replayed from one captured HIP graph of
        the whole step. Per-batch losses are summed on the device in float64 (the
        reference's Python-float sum, same order) and read once per epoch; the NaN
        check is per epoch (the reference checks every batch)."""
        from recbole_amd.trainer.graph_step import GraphedTrainStep
        gs = getattr(self, '_graph_step', None)
        if gs is None or gs.model is not self.model or gs.opt is not self.optimizer:
            gs = self._graph_step = GraphedTrainStep(self.model, self.optimizer)
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        n = 0
        for interaction in train_data:
            total.add_(gs.step(interaction.to(self.device)))
            n += 1
        self._sync_params()
        if n == 0:
            return None
        v = float(total.item())
        if np.isnan(v):
            raise ValueError('Training loss is nan')
        return v

    def _valid_epoch(self, valid_data, show_progress=False):
        valid_result = self.evaluate(valid_data, load_best_model=False, show_progress=show_progress)
        return calculate_valid_score(valid_result, self.valid_metric), valid_result

    def _sync_params(self):
        if isinstance(self.optimizer, FusedAdam):
            self.optimizer.flush()

    def _save_checkpoint(self, epoch):
        self._sync_params()
        cfg = (dict(self.config.final_config_dict) if hasattr(self.config, 'final_config_dict')
               else dict(self.config))
        state = {
            'config': _plain_config(cfg),
            'epoch': epoch,
            'cur_step': int(self.cur_step),
            'best_valid_score': float(self.best_valid_score),
            'state_dict': self.model.state_dict(),
            'optimizer': self.optimizer.state_dict(),
        }
        torch.save(state, self.saved_model_file)

    def resume_checkpoint(self, resume_file):
        checkpoint = _load_checkpoint(resume_file)
        self.start_epoch = checkpoint['epoch'] + 1
        self.cur_step = checkpoint['cur_step']
        self.best_valid_score = checkpoint['best_valid_score']
        if checkpoint['config']['model'].lower() != self.config['model'].lower():
            self.logger.warning('Architecture configuration given in config file is different '
                                'from that of checkpoint. This may yield an exception while '
                                'state_dict is being loaded.')
        self.model.load_state_dict(checkpoint['state_dict'])
        self.optimizer.load_state_dict(checkpoint['optimizer'])
        self.logger.info(f'Checkpoint loaded. Resume training from epoch {self.start_epoch}')

    def _check_nan(self, loss):
        if torch.isnan(loss):
            raise ValueError('Training loss is nan')

    def _generate_train_loss_output(self, epoch_idx, s_time, e_time, losses):
        des = self.config['loss_decimal_place'] or 4
        out = (set_color('epoch %d training', 'green') + ' [' + set_color('time', 'blue') +
               ': %.2fs, ') % (epoch_idx, e_time - s_time)
        if isinstance(losses, tuple):
            fmt = set_color('train_loss%d', 'blue') + ': %.' + str(des) + 'f'
            out += ', '.join(fmt % (i + 1, l) for i, l in enumerate(losses))
        else:
            out += set_color('train loss', 'blue') + ': ' + ('%.' + str(des) + 'f') % losses
        return out + ']'

    def fit(self, train_data, valid_data=None, verbose=True, saved=True, show_progress=False,
            callback_fn=None):
        if saved and self.start_epoch >= self.epochs:
            self._save_checkpoint(-1)
        for epoch_idx in range(self.start_epoch, self.epochs):
            t0 = time()
            train_loss = self._train_epoch(train_data, epoch_idx, show_progress=show_progress)
            self.train_loss_dict[epoch_idx] = sum(train_loss) if isinstance(train_loss, tuple) \
                else train_loss
            t1 = time()
            if verbose:
                self.logger.info(self._generate_train_loss_output(epoch_idx, t0, t1, train_loss))
            if self.eval_step <= 0 or not valid_data:
                if saved:
                    self._save_checkpoint(epoch_idx)
                    if verbose:
                        self.logger.info(set_color('Saving current', 'blue') +
                                         f': {self.saved_model_file}')
                continue
            if (epoch_idx + 1) % self.eval_step == 0:
                v0 = time()
                valid_score, valid_result = self._valid_epoch(valid_data, show_progress)
                self.best_valid_score, self.cur_step, stop_flag, update_flag = early_stopping(
                    valid_score, self.best_valid_score, self.cur_step,
                    max_step=self.stopping_step, bigger=self.valid_metric_bigger)
                v1 = time()
                if verbose:
                    self.logger.info((set_color('epoch %d evaluating', 'green') + ' [' +
                                      set_color('time', 'blue') + ': %.2fs, ' +
                                      set_color('valid_score', 'blue') + ': %f]') %
                                     (epoch_idx, v1 - v0, valid_score))
                    self.logger.info(set_color('valid result', 'blue') + ': \n' +
                                     dict2str(valid_result))
                if update_flag:
                    if saved:
                        self._save_checkpoint(epoch_idx)
                        if verbose:
                            self.logger.info(set_color('Saving current best', 'blue') +
                                             f': {self.saved_model_file}')
                    self.best_valid_result = valid_result
                if callback_fn:
                    callback_fn(epoch_idx, valid_score)
                if stop_flag:
                    if verbose:
                        self.logger.info('Finished training, best eval result in epoch %d' %
                                         (epoch_idx - self.cur_step * self.eval_step))
                    break
        return self.best_valid_score, self.best_valid_result

    # ------------------------------------------------------------------ evaluation
    def _full_sort_batch_eval(self, batched_data):
        """trainer.py:328-353 (generic path)."""
        interaction, history_index, swap_row, swap_col_after, swap_col_before = batched_data
        try:
            scores = self.model.full_sort_predict(interaction.to(self.device))
        except NotImplementedError:
            new_inter = interaction.to(self.device).repeat_interleave(self.tot_item_num)
            bs = len(new_inter)
            new_inter.update(self.item_tensor[:bs])
            scores = self.model.predict(new_inter) if bs <= self.test_batch_size else \
                self._spilt_predict(new_inter, bs)
        scores = scores.view(-1, self.tot_item_num)
        scores[:, 0] = -np.inf
        if history_index is not None:
            hr, hc = history_index
            scores[hr.to(scores.device), hc.to(scores.device)] = -np.inf
        swap_row = swap_row.to(scores.device)
        a = swap_col_after.to(scores.device)
        b = swap_col_before.to(scores.device)
        scores[swap_row, a] = scores[swap_row, b]
        return interaction, scores

    @torch.no_grad()
    def evaluate(self, eval_data, load_best_model=True, model_file=None, show_progress=False):
        if not eval_data:
            return
        if load_best_model:
            checkpoint_file = model_file or self.saved_model_file
            checkpoint = _load_checkpoint(checkpoint_file)
            self.model.load_state_dict(checkpoint['state_dict'])
            self.logger.info(f'Loading model structure and parameters from {checkpoint_file}')
        self._sync_params()
        self.model.eval()
        topk = self.evaluator.topk_evaluator
        if (eval_data.dl_type == DataLoaderType.FULL and self.config['fused_eval'] is not False
                and hasattr(self.model, 'fused_user_vectors')
                and topk is not None and len(self.evaluator.evaluators) == 1
                and self.model.fused_item_table().is_cuda):
            return fused_full_sort_eval(self.model, eval_data, topk, dp=self._dp)
        if (eval_data.dl_type == DataLoaderType.FULL and self.config['fused_eval'] is not False
                and hasattr(self.model, 'fused_query_vectors')
                and topk is not None and len(self.evaluator.evaluators) == 1
                and self.model.fused_item_table().is_cuda):
            return fused_seq_full_sort_eval(self.model, eval_data, topk)
        if (isinstance(eval_data, SequentialNegSampleDataLoader)
                and eval_data.user_inter_in_one_batch and self.config['fused_eval'] is not False
                and isinstance(eval_data.sampler, RepeatableSampler)
                and hasattr(self.model, 'fused_query_vectors')
                and topk is not None and len(self.evaluator.evaluators) == 1
                and self.model.fused_item_table().is_cuda):
            return fused_seq_sampled_eval(self.model, eval_data, topk)
        if (isinstance(eval_data, GeneralNegSampleDataLoader) and eval_data.user_inter_in_one_batch
                and eval_data.dl_format == InputType.POINTWISE
                and self.config['fused_eval'] is not False
                and hasattr(self.model, 'fused_user_vectors')
                and self.model.fused_item_table().is_cuda):
            return fused_general_sampled_eval(self.model, eval_data, self.evaluator)
        if eval_data.dl_type == DataLoaderType.FULL:
            if self.item_tensor is None:
                self.item_tensor = eval_data.get_item_feature().to(self.device).repeat(eval_data.step)
            self.tot_item_num = eval_data.dataset.item_num
        batch_matrix_list = []
        for batched_data in eval_data:
            if eval_data.dl_type == DataLoaderType.FULL:
                interaction, scores = self._full_sort_batch_eval(batched_data)
            else:
                interaction = batched_data
                bs = interaction.length
                scores = self.model.predict(interaction.to(self.device)) \
                    if bs <= self.test_batch_size else self._spilt_predict(interaction, bs)
            batch_matrix_list.append(self.evaluator.collect(interaction, scores))
        return self.evaluator.evaluate(batch_matrix_list, eval_data)

    def _spilt_predict(self, interaction, batch_size):
        from recbole_amd.data.interaction import Interaction
        split = {k: t.split(self.test_batch_size, dim=0) for k, t in interaction.interaction.items()}
        n = (batch_size + self.test_batch_size - 1) // self.test_batch_size
        out = []
        for i in range(n):
            cur = Interaction({k: v[i] for k, v in split.items()})
            r = self.model.predict(cur.to(self.device))
            out.append(r.unsqueeze(0) if r.dim() == 0 else r)
        return torch.cat(out, dim=0)


def _plain_config(cfg):
    """The config as plain Python values (enums by name, devices and other objects
    as strings): checkpoints then load with torch.load(weights_only=True)."""
    import enum

    def plain(v):
        if isinstance(v, enum.Enum):
            return v.name
        if isinstance(v, np.generic):              # numpy scalars pickle as numpy objects
            return v.item()
        if isinstance(v, (str, int, float, bool)) or v is None:
            return v
        if isinstance(v, (list, tuple)):
            return [plain(x) for x in v]
        if isinstance(v, dict):
            return {str(k): plain(x) for k, x in v.items()}
        return str(v)
    return {str(k): plain(v) for k, v in cfg.items()}


def _load_checkpoint(path):
    """torch.load without unpickling arbitrary objects (tensors, plain containers
    and numbers only), so a user-supplied .pth cannot run code on load."""
    return torch.load(str(path), map_location='cpu', weights_only=True)
