"""Drop-in ``SemanticSegmentation`` facade (code/system_factory.py).

Same constructor ``SemanticSegmentation(input_fns, model_fn, settings)``, same settings
post-processing (problem definition, ``output_Nclasses``, learning-rate boundaries in
epochs -> steps, defaults and validation), ``.train()`` runs the step loop on the native
path. Data parallelism is one process per GPU (``torch.distributed``, backend 'nccl' =
RCCL): ``train.py ... --distribute`` starts one rank per visible GPU itself (or runs as one
rank of an external ``torchrun`` launch). ``.predict()``/``.evaluate()``
(inference, visualisation, eval with moving-statistics BN) are out of scope.

Checkpoints are ``<log_dir>/model.ckpt-<step>.pt`` state dicts (named parameters, momentum,
moving statistics, EMA, global step); the training loop resumes from the latest one.
"""
from __future__ import annotations

import collections
import copy
import functools
import glob
import json
import os
import re
import time
from os.path import exists, isdir, join, split

from estimator.define_estimator_hierarchical import (define_estimator,
                                                      get_or_create_global_step, world_size)
from estimator.mode_keys import ModeKeys
from utils.utils import _replacevoids, print_metrics_from_confusion_matrix  # noqa: F401

__version__ = '0.9-mi355x'


class DistributeConfig(object):
    def __init__(self, num_towers):
        self.num_towers = num_towers


class RunConfig(object):
    """The parts of tf.estimator.RunConfig the hot path reads (input_pipelines/utils.py:119)."""

    def __init__(self, model_dir=None, save_summary_steps=120, save_checkpoints_steps=None,
                 train_distribute=None, log_step_count_steps=120):
        self.model_dir = model_dir
        self.save_summary_steps = save_summary_steps
        self.save_checkpoints_steps = save_checkpoints_steps
        self.train_distribute = train_distribute
        self.log_step_count_steps = log_step_count_steps


class SemanticSegmentation(object):

    def __init__(self, input_fns, model_fn, settings):
        assert settings is not None, 'settings must be provided for now.'
        self._settings = copy.deepcopy(settings)
        s = self._settings
        s.height_network = s.height_feature_extractor
        s.width_network = s.width_feature_extractor
        with open(s.training_problem_def_path, 'r') as fp:
            s.training_problem_def = json.load(fp)
        _set_defaults(s)
        _validate_settings(s)
        self._input_fns = input_fns
        self._model_fn = model_fn
        lids2cids = s.training_problem_def['lids2cids']
        s.lids_training_contain_unlabeled = -1 in lids2cids
        s.output_Nclasses = (max(lids2cids) + 1 +
                             (s.lids_training_contain_unlabeled or getattr(s, 'train_void_class', False)))
        self._estimator_fn = functools.partial(define_estimator, model_fn=self._model_fn)

    @property
    def settings(self):
        return self._settings

    # system_factory.py:189-302
    def _prepare_train_settings(self):
        s = self._settings
        s.num_examples_per_epoch = int(s.Ntrain * s.height_network // s.height_feature_extractor *
                                       s.width_network // s.width_feature_extractor)
        s.num_batches_per_epoch = int(s.num_examples_per_epoch / s.Nb)
        s.num_training_steps = int(s.Ne * s.num_batches_per_epoch)
        if s.learning_rate_schedule == 'piecewise_constant':
            if not (s.learning_rate_decay or s.learning_rate_values):
                s.learning_rate_decay = 0.5
            last_boundary = s.Ne - s.learning_rate_boundaries[-1]
            if last_boundary == 0:
                s.learning_rate_boundaries.pop()
            elif last_boundary < 0:
                raise ValueError('Ne is less than learning rate boundaries.')
            s.learning_rate_boundaries_epochs = s.learning_rate_boundaries
            s.learning_rate_boundaries = [lrb * s.num_batches_per_epoch
                                          for lrb in s.learning_rate_boundaries]
            if s.learning_rate_decay:
                n = len(s.learning_rate_boundaries) + 1
                s.learning_rate_values = [s.learning_rate_initial * s.learning_rate_decay ** i
                                          for i in range(n)]
        if s.distribute:
            s.ema_decay = 0
        if not s.save_checkpoints_steps:
            s.save_checkpoints_steps = s.num_batches_per_epoch

    def train(self, max_steps=None, log_fn=print, timing_warmup=None):
        """The training loop (system_factory.py:189-302). `timing_warmup` = w: after the w-th
        step of this call the device is synchronised and a clock starts; it stops after a final
        synchronisation, and ``self.last_train_timing`` = {'steps', 'seconds', 'images'} of the
        steps in between (throughput of the whole drop-in path, input pipeline included)."""
        return self._train(max_steps, log_fn, timing_warmup)

    def _train(self, max_steps, log_fn, timing_warmup):
        import torch
        s = self._settings
        self._prepare_train_settings()
        if s.distribute:
            # one process per GPU (train.main starts them when no launcher did, utils/launch.py);
            # SEG_TRAIN_BACKEND=gloo rehearses N ranks on fewer GPUs (RCCL cannot share one)
            import torch.distributed as dist
            from utils.launch import rank_device
            backend = os.environ.get('SEG_TRAIN_BACKEND', 'nccl' if torch.cuda.is_available() else 'gloo')
            torch.cuda.set_device(rank_device(int(os.environ.get('LOCAL_RANK', 0)), backend,
                                              torch.cuda.device_count()))
            if not dist.is_initialized():
                dist.init_process_group(backend=backend)
        rank = int(os.environ.get('RANK', 0))
        os.makedirs(s.log_dir, exist_ok=True)
        if rank == 0:
            settings_filename = join(s.log_dir, 'settings.txt')
            assert not exists(settings_filename), (
                f"Previous settings.txt found in {s.log_dir}. Rename or delete it manually and "
                "restart training.")
            d = collections.OrderedDict(sorted((k, v) for k, v in vars(s).items()
                                               if k != 'training_problem_def'))
            with open(settings_filename, 'w') as f:
                for k, v in enumerate(d):
                    print(f"{k:2} : {v} : {d[v]}", file=f)
        n = world_size()
        config = RunConfig(model_dir=s.log_dir, save_summary_steps=s.save_summaries_steps,
                           save_checkpoints_steps=s.save_checkpoints_steps,
                           train_distribute=DistributeConfig(n) if n > 1 else None)
        step = get_or_create_global_step()
        total = s.num_training_steps if max_steps is None else min(max_steps, s.num_training_steps)
        data = iter(self._input_fns['train'](config, s))
        from models.resnet50_extended_model_hierarchical import get_context
        ctx = get_context(config, s)
        self._maybe_restore(ctx, step)
        if rank == 0:
            log_fn(f"training {total} steps on {n} GPU(s)")
        t0 = time.time()
        first, t_timed = step.value, None
        self.last_train_timing = None
        while step.value < total:
            if timing_warmup is not None and step.value - first == timing_warmup:
                torch.cuda.synchronize()
                t_timed, s_timed = time.perf_counter(), step.value
            features, labels = next(data)
            spec = self._estimator_fn(ModeKeys.TRAIN, features, labels, config=config, params=s)
            ctx = spec.predictions['_context']
            losses = spec.train_op()
            # every rank logs its own loss terms (rank r > 0 tagged: under train.py's own
            # launch its stdout is <log_dir>/rank<r>.log)
            if step.value % s.save_summaries_steps == 0 or step.value == total:
                torch.cuda.synchronize()
                log_fn(f"{f'[rank {rank}] ' if rank else ''}step {step.value}: total {float(losses['total']):.4f} "
                       f"l1 {float(losses['l1_segmentation']):.4f} "
                       f"l2v {float(losses['l2_vehicle_segmentation']):.4f} "
                       f"l2h {float(losses['l2_human_segmentation']):.4f} "
                       f"({(time.time() - t0) / max(step.value, 1):.3f} s/step)")
            if rank == 0 and step.value % s.save_checkpoints_steps == 0:
                self.save(ctx, step.value)
        if t_timed is not None:
            torch.cuda.synchronize()
            n = step.value - s_timed
            self.last_train_timing = {'steps': n, 'seconds': time.perf_counter() - t_timed,
                                      'images': n * int(features['proimages'].shape[0])}
        if rank == 0 and ctx is not None:
            self.save(ctx, step.value)
        return step.value

    # ---- checkpoints ---------------------------------------------------------------
    def save(self, ctx, global_step):
        import torch
        # tensors, not numpy arrays: the checkpoint must load with torch.load(weights_only=True)
        named = lambda buf: {k: torch.from_numpy(v) for k, v in ctx.named(buf).items()}
        state = {'global_step': global_step, 'params': named('params'),
                 'momentum': named('momentum')}
        if ctx.ema is not None:
            state['ema'] = named('ema')
        torch.save(state, join(self._settings.log_dir, f'model.ckpt-{global_step}.pt'))
        if getattr(self._settings, 'tf_checkpoints', False):
            # the reference's Saver layout: <log_dir>/model.ckpt-<step>.{index,data-*}
            from utils.tf_checkpoint import export_checkpoint
            export_checkpoint(ctx, join(self._settings.log_dir, f'model.ckpt-{global_step}'),
                              global_step)

    def _maybe_restore(self, ctx, step):
        import torch
        ck = sorted(glob.glob(join(self._settings.log_dir, 'model.ckpt-*.pt')),
                    key=lambda p: int(re.findall(r'-(\d+)\.pt$', p)[0]))
        if not ck:
            tf_ck = sorted(glob.glob(join(self._settings.log_dir, 'model.ckpt-*.index')),
                           key=lambda p: int(re.findall(r'-(\d+)\.index$', p)[0]))
            if tf_ck:   # continue from a TF-format checkpoint in log_dir
                from utils.tf_checkpoint import import_checkpoint
                step.value = import_checkpoint(ctx, tf_ck[-1][:-len('.index')])
            elif getattr(self._settings, 'init_ckpt_path', ''):
                # define_initializers.replace_initializers: warm start (e.g. ImageNet)
                from utils.tf_checkpoint import warm_start
                warm_start(ctx, self._settings.init_ckpt_path,
                           psp_module=bool(getattr(self._settings, 'psp_module', False)))
            return
        state = torch.load(ck[-1], weights_only=True)
        ctx.load_params(state['params'])   # (also resets the EMA shadows to the weights)
        for buf, saved in ((ctx.momentum, state['momentum']), (ctx.ema, state.get('ema'))):
            if buf is None or saved is None:
                continue
            for p in ctx.param_info:
                if p.name in saved:
                    buf[p.offset:p.offset + p.numel].copy_(torch.as_tensor(saved[p.name]).reshape(-1))
        step.value = int(state['global_step'])

    # ---- evaluation / prediction (system_factory.py:148-158,304-412) -------------------
    def _cid_maps(self):
        s = self._settings
        tcids = list(range(s.output_Nclasses))
        if s.lids_training_contain_unlabeled and not getattr(s, 'train_void_class', False):
            tcids[-1] = -1   # ignore void if it was not trained
        path = getattr(s, 'evaluation_problem_def_path', None)
        if path:
            with open(path, 'r') as fp:
                s.evaluation_problem_def = json.load(fp)
        else:
            s.evaluation_problem_def = s.training_problem_def
        s.training_cids2evaluation_cids = s.evaluation_problem_def.get(
            'training_cids2evaluation_cids', list(tcids))
        path = getattr(s, 'inference_problem_def_path', None)
        if path:
            with open(path, 'r') as fp:
                s.inference_problem_def = json.load(fp)
        else:
            s.inference_problem_def = s.training_problem_def
        s.training_cids2inference_cids = s.inference_problem_def.get(
            'training_cids2inference_cids', list(tcids))

    def _checkpoints(self):
        """Checkpoint paths in log_dir, oldest first: the native ``model.ckpt-<step>.pt``
        files, else the TF V2 prefixes ``model.ckpt-<step>`` (the reference's Saver layout)."""
        s = self._settings
        ck = sorted(glob.glob(join(s.log_dir, 'model.ckpt-*.pt')),
                    key=lambda p: int(re.findall(r'-(\d+)\.pt$', p)[0]))
        if not ck:
            ck = [p[:-len('.index')] for p in sorted(
                glob.glob(join(s.log_dir, 'model.ckpt-*.index')),
                key=lambda p: int(re.findall(r'-(\d+)\.index$', p)[0]))]
        return ck

    def _restore_for_eval(self, ctx, ckpt_path):
        import torch
        s = self._settings
        if not ckpt_path:
            ck = self._checkpoints()
            if not ck:   # tf.estimator: "Could not find trained model in model_dir"
                raise ValueError(f'Could not find a trained model (model.ckpt-*.pt or a TF '
                                 f'model.ckpt-*.index) in log_dir {s.log_dir}')
            ckpt_path = ck[-1]
        restore_emas = bool(getattr(s, 'restore_emas', False))
        if exists(ckpt_path + '.index'):
            from utils.tf_checkpoint import import_checkpoint
            return import_checkpoint(ctx, ckpt_path, momentum=False, restore_emas=restore_emas)
        if not exists(ckpt_path):
            raise ValueError(f'checkpoint {ckpt_path} not found (neither a .pt file nor a TF '
                             f'prefix with {ckpt_path}.index)')
        state = torch.load(ckpt_path, weights_only=True)
        if restore_emas and 'ema' not in state:
            raise KeyError(f'--restore_emas: {ckpt_path} holds no EMA shadows (trained with '
                           f'--ema_decay 0 or --distribute)')
        params = state['ema'] if restore_emas else state['params']
        ctx.load_params(params)
        if restore_emas:   # the EMA excludes the BN moving statistics (define_savers.py:46)
            ctx.load_params({k: v for k, v in state['params'].items() if 'moving_' in k})
        return int(state['global_step'])

    def evaluate(self, max_steps=None, log_fn=print):
        """One pass over the eval input per checkpoint; returns [{'global_step', 'loss',
        'confusion_matrix'}] with the void row/column dropped as the reference does."""
        import numpy as np
        import torch
        from models.resnet50_extended_model_hierarchical import get_context
        s = self._settings
        self._cid_maps()
        s.num_examples = int(s.Neval * s.height_network // s.height_feature_extractor *
                             s.width_network // s.width_feature_extractor)
        s.num_batches_per_epoch = int(s.num_examples / s.Nb)
        s.num_eval_steps = s.num_batches_per_epoch if max_steps is None else \
            min(max_steps, s.num_batches_per_epoch)
        config = RunConfig(model_dir=s.log_dir)
        labels_names = s.evaluation_problem_def['cids2labels']
        void_exists = -1 in s.evaluation_problem_def['lids2cids']
        if void_exists and not getattr(s, 'train_void_class', False):
            labels_names = labels_names[:-1]
        ckpts = [getattr(s, 'ckpt_path', None)]
        if getattr(s, 'eval_all_ckpts', False):
            ckpts = self._checkpoints()
            if not ckpts:
                raise ValueError(f'--eval_all_ckpts: no checkpoints in log_dir {s.log_dir}')
        ctx = get_context(config, s, mode=ModeKeys.EVAL)
        all_metrics = []
        for cp in ckpts:
            gstep = self._restore_for_eval(ctx, cp)
            cm = None
            data = iter(self._input_fns['eval'](config, s))
            for _ in range(s.num_eval_steps):
                features, labels = next(data)
                spec = self._estimator_fn(ModeKeys.EVAL, features, labels, config=config,
                                          params=s)
                c = spec.eval_metric_ops['confusion_matrix'].to(torch.int64)
                cm = c if cm is None else cm + c
            cm = cm.cpu().numpy().astype(np.int32)
            if void_exists and not getattr(s, 'train_void_class', False):
                cm = cm[:-1, :-1]
            metrics = {'global_step': gstep, 'loss': 0.0, 'confusion_matrix': cm}
            print_metrics_from_confusion_matrix(np.asarray(cm), labels_names,
                                                printcmd=bool(log_fn))
            all_metrics.append(metrics)
        return all_metrics

    def predict(self, max_steps=None):
        """Generator of per-batch predictions dicts ('decisions' [N, H, W] device int32 in
        inference cids, low-res logits, and the input's raw images/paths when given)."""
        from models.resnet50_extended_model_hierarchical import get_context
        s = self._settings
        self._cid_maps()
        config = RunConfig(model_dir=s.log_dir)
        ctx = get_context(config, s, mode=ModeKeys.PREDICT)
        self._restore_for_eval(ctx, getattr(s, 'ckpt_path', None))
        for i, (features, _) in enumerate(self._input_fns['predict'](config, s)):
            if max_steps is not None and i >= max_steps:
                return
            spec = self._estimator_fn(ModeKeys.PREDICT, features, None, config=config, params=s)
            yield spec.predictions


def _set_defaults(settings):
    if getattr(settings, 'learning_rate_schedule', None) == 'piecewise_constant':
        if not (settings.learning_rate_decay or settings.learning_rate_values):
            settings.learning_rate_decay = 0.5


def _validate_settings(settings):
    assert settings.height_network == settings.height_feature_extractor and \
        settings.width_network == settings.width_feature_extractor, (
            'For now height/width_network and height/width_feature_extractor should be equal.')
    if getattr(settings, 'learning_rate_schedule', None) == 'piecewise_constant':
        if not (bool(settings.learning_rate_decay) != bool(settings.learning_rate_values)):
            raise AttributeError('If `learning_rate_schedule` is `piecewise_constant` exactly one '
                                 'of `learning_rate_decay` or `learning_rate_values` must be given.')
    lids2cids_unique = set(settings.training_problem_def['lids2cids'])
    cid_max = max(lids2cids_unique)
    lids2cids_unique.discard(-1)
    if not (lids2cids_unique == set(range(cid_max + 1))):
        raise ValueError('lids2cids field in training problem definition contains not '
                         'continuous class ids.')
