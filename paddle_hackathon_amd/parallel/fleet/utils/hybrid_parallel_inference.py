"""``fleet.utils.HybridParallelInferenceHelper`` (reference python/paddle/distributed/fleet/utils/
hybrid_parallel_inference.py:23): splits a static inference Program — typically a generation
``While`` loop whose body is cut into pipeline stages with ``device_guard("gpu:k")`` — over
``num_pp`` pipeline stages x ``num_mp`` model-parallel ranks (rank = stage * num_mp + mp index).

``gen_infer_program`` rewrites the main program in place for this rank:

* every op keeps its ``op_device`` ("gpu:k" = stage k, "gpu:all" = every stage: readers and the
  while op are marked so; any other op without one is an error, as in the reference);
* a variable produced on stage p and read on stage q gets a ``send_v2`` right after its producer
  on p and a ``recv_v2`` at the same program position on q (both walk the program in one order,
  so the point-to-point messages pair up in order — what RCCL needs, it has no tags);
* in the While body the last stage sends ``sync_in_while_var_names`` (e.g. the loop condition) to
  every other stage and ``sync_in_while_lastpp2firstpp_var_names`` (e.g. the token array the first
  stage reads next step) to the first one, right after their last writer (ahead of the reference's
  closing ``assign(cast(cond_int), cond)``);
* the ops of other stages are dropped.

Tensors travel as a [ndim, dims..., dtype] header plus the data; tensor arrays as their length
and then each element. Over RCCL between the GPUs of one node that is xGMI point-to-point."""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as tdist

from ....framework.core import _wrap
from ....static import program as P

__all__ = ["HybridParallelInferenceHelper"]

_HDR = 10
_DT = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.bool,
       torch.int8, torch.uint8, torch.int16]


def _stage(op):
    dev = op.attrs.get("op_device")
    if dev is None:
        return None
    tail = str(dev).rsplit(":", 1)[-1]
    return None if tail == "all" or ":" not in str(dev) else int(tail)


class _P2P:
    """blocking point-to-point transfers over the default process group"""

    def __init__(self, device):
        self.cpu = tdist.get_backend() == "gloo"
        self.device = device

    def _dev(self):
        return torch.device("cpu") if self.cpu else self.device

    def send_tensor(self, t, dst):
        t = t.detach().contiguous()
        t = t.cpu() if self.cpu else t.to(self.device)
        assert t.dim() <= _HDR - 2, f"send_tensor: {t.dim()} dims (the header holds at most {_HDR - 2})"
        hdr = torch.zeros(_HDR, dtype=torch.int64)
        hdr[0] = t.dim()
        hdr[1:1 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.int64)
        hdr[-1] = _DT.index(t.dtype)
        tdist.send(hdr.to(self._dev()), dst)
        if t.dtype == torch.bool:   # RCCL moves no bool: as uint8
            t = t.to(torch.uint8)
        tdist.send(t, dst)

    def recv_tensor(self, src):
        hdr = torch.zeros(_HDR, dtype=torch.int64, device=self._dev())
        tdist.recv(hdr, src)
        h = hdr.cpu().tolist()
        shape, dt = h[1:1 + h[0]], _DT[h[-1]]
        buf = torch.empty(shape, dtype=torch.uint8 if dt == torch.bool else dt, device=self._dev())
        tdist.recv(buf, src)
        return buf.to(dt).to(self.device)

    def send(self, val, dst):
        if isinstance(val, list):   # a tensor array: its length, then the elements
            self.send_tensor(torch.tensor([len(val)], dtype=torch.int64), dst)
            for v in val:
                self.send_tensor(v._t, dst)
        else:
            self.send_tensor(val._t, dst)

    def recv(self, src, is_array):
        if is_array:
            n = int(self.recv_tensor(src).reshape(-1)[0])
            return [_wrap(self.recv_tensor(src)) for _ in range(n)]
        return _wrap(self.recv_tensor(src))


class HybridParallelInferenceHelper:
    def __init__(self, startup_program, main_program, num_mp=1, num_pp=1, micro_batch_size=1, beam_size=1,
                 init_comm=True, role_maker=None):
        assert isinstance(startup_program, P.Program) and isinstance(main_program, P.Program)
        from ....framework import core as _core
        assert _core._mode.static, "Only static mode is supported."
        self._startup_program, self._main_program = startup_program, main_program
        self.micro_batch_size, self.beam_size, self.init_comm = micro_batch_size, beam_size, init_comm
        if role_maker is not None:
            self.rank, self.nranks = role_maker._worker_index(), role_maker._worker_num()
        elif tdist.is_available() and tdist.is_initialized():
            self.rank, self.nranks = tdist.get_rank(), tdist.get_world_size()
        else:
            self.rank = int(os.environ.get("PADDLE_TRAINER_ID", "0"))
            self.nranks = int(os.environ.get("PADDLE_TRAINERS_NUM", "1"))
        assert num_mp * num_pp == self.nranks, f"num_mp * num_pp = {num_mp * num_pp} != {self.nranks} ranks"
        self.num_mp, self.num_pp = num_mp, num_pp
        arr = np.arange(0, num_pp * num_mp).reshape([num_pp, num_mp])
        ipp, imp = (int(a[0]) for a in np.where(arr == self.rank))
        self.mp_group = arr[ipp, :]
        self.pp_group = arr[:, imp]
        self._stage = ipp
        self._pipeline_pair, self._pipeline_pair_in_while = [], []
        self._device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device("cpu")

    # ------------------------------------------------------------------------ rewriting
    def _var(self, ref):
        if isinstance(ref, P.Variable):
            return ref
        for b in self._main_program.blocks:
            if ref in b.vars:
                return b.vars[ref]
        for b in self._main_program.blocks:   # "cond_int.tmp_0"-style reference names: by stem
            for name, v in b.vars.items():
                if name.split(".")[0] == str(ref).split(".")[0]:
                    return v
        raise KeyError(f"variable {ref!r} not found in the main program")

    def _send_op(self, var, dst_stage, stage, xfer):
        dst = int(self.pp_group[dst_stage])

        def send_v2(x):
            xfer.send(x, dst)
            return None
        return P.OpDesc("send_v2", send_v2, (), {"x": var}, None,
                        attrs={"op_device": f"gpu:{stage}", "peer": dst, "ring_id": 0})

    def _recv_op(self, var, src_stage, stage, xfer):
        src = int(self.pp_group[src_stage])
        is_array = type(var).__name__ == "_ArrayVar"

        def recv_v2():
            return xfer.recv(src, is_array)
        op = P.OpDesc("recv_v2", recv_v2, (), {}, var, attrs={"op_device": f"gpu:{stage}", "peer": src, "ring_id": 0})
        return op

    def _insert_boundaries(self, blk, xfer):
        """send after the producer / recv at the same position, for every cross-stage read"""
        producer = {}
        done = set()
        new = []
        pending = []   # (position after which to place, op)
        for i, op in enumerate(blk.ops):
            q = _stage(op)
            if q is not None:
                for v in P._iter_vars((op.args, op.kwargs)):
                    src = producer.get(id(v))
                    if src is None:
                        continue
                    p = src[1]
                    if p is None or p == q or (id(v), q) in done:
                        continue
                    done.add((id(v), q))
                    pair = (min(p, q), max(p, q))
                    if pair not in self._pipeline_pair:
                        self._pipeline_pair.append(pair)
                    pending.append((src[0], p, q, v))
            for v in P._iter_vars(op.outputs):
                producer[id(v)] = (i, q)
        at = {}
        for pos, p, q, v in pending:
            at.setdefault(pos, []).append((p, q, v))
        for i, op in enumerate(blk.ops):
            new.append(op)
            for p, q, v in at.get(i, ()):
                if self._stage == p:
                    new.append(self._send_op(v, q, p, xfer))
                elif self._stage == q:
                    new.append(self._recv_op(v, p, q, xfer))
        blk.ops = new

    def _insert_while_sync(self, blk, last_to_first, sync_all, xfer):
        stages = sorted({_stage(op) for op in blk.ops if _stage(op) is not None})
        if len(stages) < 2:
            return
        first, last = stages[0], stages[-1]
        assert len(blk.ops) > 2, ("the While body must end with assign(cast(cond_int), cond) on every stage "
                                  "(more than 2 ops)")
        ins = []
        for q in stages:
            if q == last:
                continue
            names = list(sync_all) + (list(last_to_first) if q == first else [])
            for ref in names:
                v = self._var(ref)
                if self._stage == last:
                    ins.append(self._send_op(v, q, last, xfer))
                elif self._stage == q:
                    ins.append(self._recv_op(v, last, q, xfer))
        # right after the last op that writes a synced variable (the reference inserts in front of
        # the body's closing assign(cast(cond_int), cond) pair; its cast must read the synced value)
        want = {id(self._var(r)) for r in list(sync_all) + list(last_to_first)}
        k = max([i + 1 for i, op in enumerate(blk.ops) if any(id(v) in want for v in P._iter_vars(op.outputs))]
                or [len(blk.ops) - 2])
        blk.ops[k:k] = ins

    def _split(self, blk):
        keep = []
        for op in blk.ops:
            s = _stage(op)
            if s is None or s == self._stage:
                keep.append(op)
        blk.ops = keep

    _DEVICE_ALL = ("create_py_reader", "read", "create_double_buffer_reader", "while")

    def _add_op_device_attr(self, blk):
        """reader and while ops run on every stage ("gpu:all"), as the reference marks them
        (hybrid_parallel_inference.py:446)"""
        for op in blk.ops:
            if op.type.rsplit(".", 1)[-1] in self._DEVICE_ALL:
                op.attrs["op_device"] = "gpu:all"
            if op.type == "while":
                self._add_op_device_attr(self._main_program.blocks[op.attrs["sub_block"]])

    def _check_validation(self, blk):
        """every other op must carry its stage (reference _check_validation, :475): an op without
        op_device would be kept on every stage and fail later reading a value another stage made"""
        for op in blk.ops:
            if op.type == "while":
                self._check_validation(self._main_program.blocks[op.attrs["sub_block"]])
            dev = op.attrs.get("op_device")
            assert dev, f"{op.type} has no op_device set (use static.device_guard('gpu:k') for every op)"

    def gen_infer_program(self, sync_in_while_lastpp2firstpp_var_names=None, sync_in_while_var_names=None,
                          debug=False):
        """rewrite the main (and startup) program for this rank's pipeline stage"""
        main = self._main_program
        gblk = main.global_block()
        self._add_op_device_attr(gblk)
        self._check_validation(gblk)
        xfer = _P2P(self._device)
        self._insert_boundaries(gblk, xfer)
        whiles = [op for op in gblk.ops if op.type == "while"]
        assert len(whiles) < 2, "More than one while op found."
        if whiles:
            body = main.blocks[whiles[0].attrs["sub_block"]]
            self._insert_boundaries(body, xfer)
            self._insert_while_sync(body, sync_in_while_lastpp2firstpp_var_names or [],
                                    sync_in_while_var_names or [], xfer)
            self._split(body)
        self._split(gblk)
        self._split(self._startup_program.global_block())
        if debug:
            with open(f"main_program.txt.{self.rank}", "w") as f:
                f.write(repr(main))
        return main
