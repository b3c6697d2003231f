"""Static post-training quantization (reference: python/paddle/fluid/contrib/slim/quantization/
post_training_quantization.py:103 PostTrainingQuantization, WeightQuantization).

``PostTrainingQuantization(executor, model_dir, ...).quantize()`` loads an inference model, runs
the calibration batches through it collecting |x| statistics of every activation input of the
quantizable ops (conv2d / depthwise_conv2d / mul / matmul(_v2) / fc), computes each threshold with
``algo`` (cal_kl_threshold.Calibrator), quantizes the weights per channel and inserts frozen
quant-dequant ops with the calibrated scales (``onnx_format=True``: quantize_linear /
dequantize_linear pairs). ``save_quantized_model`` writes the result as an inference model whose
ops are reference op types.

``WeightQuantization(model_dir).quantize_weight_to_int(...)`` stores the weights of the
quantizable ops as int8 levels + per-channel scales (dequantize_linear in front of the consumer).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .....framework.core import Parameter, Tensor, _wrap
from .....static import program as P
from . import quantization_pass as QP
from .cal_kl_threshold import Calibrator

__all__ = ["PostTrainingQuantization", "WeightQuantization"]


def _prefix(model_dir, model_filename):
    if model_filename:
        base = model_filename[:-len(".pdmodel")] if model_filename.endswith(".pdmodel") else model_filename
        return os.path.join(model_dir, base)
    for cand in ("inference", "model", "__model__"):
        if os.path.exists(os.path.join(model_dir, cand + ".pdmodel")):
            return os.path.join(model_dir, cand)
    return model_dir


def _load(model_dir, model_filename, params_filename, executor):
    from ..... import static
    pre = _prefix(model_dir, model_filename)
    if os.path.exists(pre + ".pdmodel"):
        return static.load_inference_model(pre, executor)
    from .....fluid import io as fio   # 1.x directory layout (__model__ + params)
    return fio.load_inference_model(model_dir, executor, model_filename, params_filename)


def _batches(batch_generator, sample_generator, data_loader, batch_size, batch_nums, feed_names):
    n = 0
    if data_loader is not None:
        src = data_loader() if callable(data_loader) and not hasattr(data_loader, "__iter__") else data_loader
    elif batch_generator is not None:
        src = batch_generator()
    elif sample_generator is not None:
        def gen():
            buf = []
            for s in sample_generator():
                buf.append(s)
                if len(buf) == batch_size:
                    yield [np.stack([np.asarray(b[i]) for b in buf]) for i in range(len(buf[0]))]
                    buf = []
        src = gen()
    else:
        raise ValueError("PostTrainingQuantization needs a batch_generator, sample_generator or data_loader")
    for batch in src:
        if isinstance(batch, dict):
            feed = {k: (v.numpy() if isinstance(v, Tensor) else np.asarray(v)) for k, v in batch.items()}
        else:
            items = batch if isinstance(batch, (list, tuple)) else [batch]
            if len(items) == 1 and isinstance(items[0], dict):
                feed = items[0]
            else:
                feed = {name: (v.numpy() if isinstance(v, Tensor) else np.asarray(v))
                        for name, v in zip(feed_names, items)}
        yield feed
        n += 1
        if batch_nums is not None and n >= batch_nums:
            break


def _scale_param(value, name):
    p = Parameter(data=torch.as_tensor(np.asarray(value, dtype=np.float32).reshape(-1)), name=name, trainable=False)
    p.stop_gradient = True
    return p


class PostTrainingQuantization:
    def __init__(self, executor=None, model_dir=None, scope=None, model_filename=None, params_filename=None,
                 batch_generator=None, sample_generator=None, data_loader=None, batch_size=10, batch_nums=None,
                 algo="KL", hist_percent=0.99999, quantizable_op_type=("conv2d", "depthwise_conv2d", "mul"),
                 round_type="round", learning_rate=0.001, is_full_quantize=False, bias_correction=False,
                 activation_bits=8, weight_bits=8, activation_quantize_type="range_abs_max",
                 weight_quantize_type="channel_wise_abs_max", onnx_format=False, freeze_model=True,
                 optimize_model=False, is_use_cache_file=False, skip_tensor_list=None, same_scale_tensor_list=None,
                 cache_dir=None, scale_dict=None, return_graph=False, program=None, feed_list=None,
                 fetch_list=None):
        if algo not in ("KL", "hist", "avg", "mse", "emd", "abs_max", "min_max"):
            raise ValueError(f"unknown algo {algo!r}")
        if weight_quantize_type not in ("abs_max", "channel_wise_abs_max"):
            raise ValueError(f"unknown weight_quantize_type {weight_quantize_type!r}")
        from ..... import static
        self._exe = executor or static.Executor()
        self._model_dir, self._model_filename, self._params_filename = model_dir, model_filename, params_filename
        self._gens = (batch_generator, sample_generator, data_loader)
        self._batch_size, self._batch_nums = batch_size, batch_nums
        self._algo, self._percent = algo, hist_percent
        self._types = tuple(QP.QUANT_OPS) if is_full_quantize else tuple(quantizable_op_type)
        self._abits, self._wbits = activation_bits, weight_bits
        self._wtype = weight_quantize_type
        self._onnx = onnx_format
        self._skip = set(skip_tensor_list or [])
        self._same = [list(g) for g in (same_scale_tensor_list or [])]
        self._scale_dict = dict(scale_dict or {})
        self._program = program
        self._feed_names = feed_list
        self._fetch = fetch_list
        self._thresholds = {}
        self._return_graph = return_graph

    # ------------------------------------------------------------------------------ steps
    def _load_model(self):
        if self._program is None:
            self._program, self._feed_names, self._fetch = _load(self._model_dir, self._model_filename,
                                                                 self._params_filename, self._exe)
        if self._feed_names and not isinstance(self._feed_names[0], str):
            self._feed_names = [v.name for v in self._feed_names]

    def _targets(self):
        """the activation Variables feeding quantizable ops (by identity, program order)"""
        seen, out = set(), []
        for op, act, w, axis in QP._quantizable(self._program, self._types):
            v = op.kwargs[act]
            if isinstance(v, P.Variable) and v.name not in self._skip and id(v) not in seen:
                seen.add(id(v))
                out.append(v)
        return out

    def _sample(self, targets):
        cals = {id(v): Calibrator(self._algo, self._abits, self._percent) for v in targets}
        for feed in _batches(*self._gens, self._batch_size, self._batch_nums, self._feed_names):
            vals = self._exe.run(self._program, feed=feed, fetch_list=list(targets))
            for v, val in zip(targets, vals):
                cals[id(v)].update(val.numpy() if isinstance(val, Tensor) else np.asarray(val))
        for v in targets:
            self._thresholds[v.name] = float(self._scale_dict.get(v.name, cals[id(v)].threshold()))
        for group in self._same:   # tensors that must share one scale (concat inputs ...)
            m = max((self._thresholds.get(n, 0.0) for n in group), default=0.0)
            for n in group:
                if n in self._thresholds:
                    self._thresholds[n] = m

    def _insert(self, targets):
        blk = self._program.global_block()
        QO = QP._qo()
        acts = {}
        wdone = {}
        from .....ops import quant as Q
        for op, act, w, axis in QP._quantizable(self._program, self._types):
            v = op.kwargs[act]
            if isinstance(v, P.Variable) and v.name in self._thresholds:
                if id(v) not in acts:
                    s = _scale_param(self._thresholds[v.name], v.name + ".quant_scale")
                    if self._onnx:
                        d, pair = QP._pair(blk, v, s, self._abits, -1)
                        for o in pair:
                            QP._insert_before(blk, op, o)
                    else:
                        d = QP._new_var(blk, v, v.name + ".quantized.dequantized")
                        QP._insert_before(blk, op, QP._make_op(
                            "fake_quantize_dequantize_fixed_scale", {"x": v, "scale": s, "bit_length": self._abits},
                            d))
                    acts[id(v)] = d
                QP._replace_input(op, act, acts[id(v)])
            if w is None or not QP._is_weight(op.kwargs[w]):
                continue
            wt = op.kwargs[w]
            if id(wt) not in wdone:
                ax = axis if self._wtype == "channel_wise_abs_max" else None
                sc = Q.channel_abs_max(wt._t, ax) if ax is not None else Q.abs_max(wt._t)
                sp = _scale_param(sc.cpu().numpy(), (wt.name or "w") + ".quant_scale")
                sp._t = sp._t.to(wt._t.device)
                if self._onnx:
                    d, pair = QP._pair(blk, wt, sp, self._wbits, ax if ax is not None else -1)
                    for o in pair:
                        QP._insert_before(blk, op, o)
                else:
                    d = QP._new_var(blk, _wrap(wt._t.to("meta")), (wt.name or "w") + ".quantized.dequantized")
                    QP._insert_before(blk, op, QP._make_op(
                        "fake_quantize_dequantize_fixed_scale",
                        {"x": wt, "scale": sp, "bit_length": self._wbits, "quant_axis": ax}, d))
                wdone[id(wt)] = d
            QP._replace_input(op, w, wdone[id(wt)])

    def quantize(self):
        """calibrate and insert the quantization ops -> the quantized Program"""
        self._load_model()
        targets = self._targets()
        self._sample(targets)
        self._insert(targets)
        if self._return_graph:
            return QP.IrGraph(self._program, for_test=True)
        return self._program

    def save_quantized_model(self, save_model_path, model_filename=None, params_filename=None):
        from ..... import static
        blk = self._program.global_block()
        feeds = [blk.vars[n] for n in self._feed_names]
        pre = os.path.join(save_model_path, (model_filename or "model.pdmodel").replace(".pdmodel", ""))
        static.save_inference_model(pre, feeds, list(self._fetch), self._exe, program=self._program)
        return pre

    @property
    def thresholds(self):
        return dict(self._thresholds)


class WeightQuantization:
    """int8 (or int16) storage of the weights of the quantizable ops of an inference model"""
    _supported_quantizable_op_type = ("conv2d", "depthwise_conv2d", "mul", "matmul_v2", "fc")

    def __init__(self, model_dir, model_filename=None, params_filename=None):
        self._model_dir, self._model_filename, self._params_filename = model_dir, model_filename, params_filename

    def quantize_weight_to_int(self, save_model_dir, save_model_filename=None, save_params_filename=None,
                               quantizable_op_type=("conv2d", "mul"), weight_bits=8,
                               weight_quantize_type="channel_wise_abs_max", generate_test_model=False,
                               threshold_rate=0.0):
        from ..... import static
        exe = static.Executor()
        prog, feeds, fetches = _load(self._model_dir, self._model_filename, self._params_filename, exe)
        QP.ConvertToInt8Pass(quantizable_op_type=quantizable_op_type, weight_bits=weight_bits).apply(prog)
        blk = prog.global_block()
        feed_vars = [blk.vars[n] if isinstance(n, str) else n for n in feeds]
        pre = os.path.join(save_model_dir, (save_model_filename or "model.pdmodel").replace(".pdmodel", ""))
        static.save_inference_model(pre, feed_vars, list(fetches), exe, program=prog)
        return pre

    def convert_weight_to_fp16(self, save_model_dir):
        from ..... import static
        exe = static.Executor()
        prog, feeds, fetches = _load(self._model_dir, self._model_filename, self._params_filename, exe)
        for p in prog.all_parameters():
            if p._t.is_floating_point():
                p._t = p._t.half().float()
        blk = prog.global_block()
        static.save_inference_model(os.path.join(save_model_dir, "model"), [blk.vars[n] for n in feeds],
                                    list(fetches), exe, program=prog)
