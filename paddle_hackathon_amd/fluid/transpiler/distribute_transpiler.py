"""``DistributeTranspiler``: rewrite a single-process static training Program into trainer and
parameter-server Programs (reference: python/paddle/fluid/transpiler/distribute_transpiler.py —
transpile :258 (param/grad blocks, send / recv insertion), get_pserver_program :1045
(listen_and_serv + per-block optimize blocks), get_startup_program :1180; ps_dispatcher.py).

What the rewrite does, the reference's way:

* every trainable parameter (and its gradient) is cut into row blocks (``slice_var_up``: up to one
  block per server, each >= ``min_block_size`` elements, whole rows) that ``split_method``
  (RoundRobin / HashName) places on the server endpoints;
* trainer program: the optimizer op is removed; per parameter a ``send`` op pushes the gradient's
  blocks to their servers, a ``send_barrier`` closes the step (sync mode), per parameter a ``recv``
  op pulls the updated blocks back into the parameter and a ``fetch_barrier`` ends the step;
* pserver program: one ``listen_and_serv`` op that serves this endpoint's blocks until every
  trainer has called ``Executor.close()``; the blocks' optimizer (SGD / Adam / Adagrad with the
  trainer program's learning rate) runs inside the server;
* ``config.mode == "nccl2"`` / ``"collective"``: no servers — the gradients are summed over the
  trainers with one coalesced all-reduce before the optimizer op and the parameters broadcast from
  trainer 0 by the startup program (torch.distributed must be initialised, RCCL on GPUs).

MI355X-first differences: the server is the native C++ table server (``csrc/runtime/ps.cpp``,
parallel/ps) rather than a Program interpreter, so a pserver program carries no optimizer ops —
the rule, learning rate and Adam / Adagrad state are the table's. In sync mode the server
averages the trainers' gradients (the reference's sum + scale 1/trainers) and applies the update
once; ``recv`` waits for that version. Learning-rate schedules and regularisers of the origin
program are not transpiled (constant learning rate on the servers)."""
from __future__ import annotations

import math
import zlib

import numpy as np
import torch

__all__ = ["DistributeTranspiler", "DistributeTranspilerConfig", "HashName", "RoundRobin"]

_RULES = {"sgd": "sgd", "adam": "adam", "adagrad": "adagrad"}


class DistributeTranspilerConfig:
    """reference DistributeTranspilerConfig: slicing, placement and mode switches"""

    def __init__(self):
        self.slice_var_up = True
        self.split_method = None
        self.min_block_size = 8192
        self.enable_dc_asgd = False
        self.mode = "pserver"
        self.print_log = False
        self.wait_port = True
        self.runtime_split_send_recv = False
        self.sync_mode = True
        self.geo_sgd_mode = False
        self.geo_sgd_need_push_nums = 100
        self.nccl_comm_num = 1
        self.use_hierarchical_allreduce = False
        self.hierarchical_allreduce_inter_nranks = 0
        self.collective_mode = None


class PSDispatcher:
    def __init__(self, pserver_endpoints):
        self._eps = list(pserver_endpoints)

    @property
    def eps(self):
        return self._eps

    def reset(self):
        pass


class HashName(PSDispatcher):
    """block -> endpoint by a hash of the block name (crc32: the same on every process, unlike the
    salted built-in ``hash``)"""

    def dispatch(self, varlist):
        return [self._eps[zlib.crc32(v.name.encode()) % len(self._eps)] for v in varlist]


class RoundRobin(PSDispatcher):
    def __init__(self, pserver_endpoints):
        super().__init__(pserver_endpoints)
        self._i = 0

    def dispatch(self, varlist):
        out = []
        for _ in varlist:
            out.append(self._eps[self._i % len(self._eps)])
            self._i += 1
        return out

    def reset(self):
        self._i = 0


class VarBlock:
    """rows [row0, row1) of parameter ``param`` (flattened elements [offset, offset + numel))"""

    def __init__(self, param, idx, row0, row1, row_numel):
        self.param, self.idx, self.row0, self.row1 = param, idx, row0, row1
        self.offset, self.numel = row0 * row_numel, (row1 - row0) * row_numel
        self.name = f"{param.name}.block{idx}"
        self.endpoint = None
        self.table = None

    def __repr__(self):
        return f"{self.name}:{self.offset}:{self.numel}@{self.endpoint}"


def slice_variable(param, slice_count, min_block_size):
    """the reference's slice_variable: at most ``slice_count`` blocks of whole rows, each at least
    ``min_block_size`` elements"""
    shape = list(param.shape) or [1]
    numel = int(np.prod(shape))
    rows = shape[0]
    row_numel = numel // rows if rows else 1
    split = max(1, min(slice_count, numel // max(1, min_block_size)))
    rows_per_block = max(1, math.ceil(rows / split))
    blocks = []
    r = 0
    while r < rows:
        blocks.append(VarBlock(param, len(blocks), r, min(rows, r + rows_per_block), row_numel))
        r += rows_per_block
    return blocks


class _TrainerSession:
    """trainer-side connection state that the transpiled program's send / recv ops share"""

    def __init__(self, t):
        self.t = t
        self.clients = None
        self.step = 0
        self.closed = False

    def _connect(self):
        from ...parallel.ps import PSClient
        t = self.t
        self.clients = {ep: PSClient([ep]) for ep in t.pserver_endpoints}
        self.ctl = self.clients[t.pserver_endpoints[0]]   # barriers are served by the first server
        if t.trainer_id == 0:
            for blk in t.blocks:
                init = blk.param._t.detach().reshape(-1)[blk.offset:blk.offset + blk.numel].float().cpu().numpy()
                self.clients[blk.endpoint].create_dense(
                    blk.table, blk.numel, rule=t.rule, lr=t.lr, init=init,
                    sync_trainers=t.trainers if t.sync_mode else 1, **t.rule_kw)
        else:
            for blk in t.blocks:   # same table geometry, no (re)initialisation
                self.clients[blk.endpoint]._dense[blk.table] = (blk.numel, [(0, blk.numel)])
        self.ctl.barrier(t.trainers, tag=1)
        for p in t.params:         # every trainer starts from trainer 0's values
            self._pull(p, 0)

    def _pull(self, p, min_version):
        buf = np.empty(p._t.numel(), np.float32)
        for blk in self.t.by_param[p.name]:
            self.clients[blk.endpoint].pull_dense(blk.table, out=buf[blk.offset:blk.offset + blk.numel],
                                                  min_version=min_version)
        with torch.no_grad():
            p._t.copy_(torch.from_numpy(buf).reshape(p._t.shape).to(p._t.device, p._t.dtype))

    def send(self, param, grad):
        if self.clients is None:
            self._connect()
        g = grad._t.detach().reshape(-1).float().cpu().numpy()
        for blk in self.t.by_param[param.name]:
            self.clients[blk.endpoint].push_dense(blk.table, g[blk.offset:blk.offset + blk.numel])

    def recv(self, param):
        self._pull(param, self.step if self.t.sync_mode else 0)

    def close(self):
        if self.closed or self.clients is None:
            return
        self.closed = True
        self.ctl.barrier(self.t.trainers, tag=1 << 20)
        if self.t.trainer_id == 0:
            for c in self.clients.values():
                c.stop_servers()
        for c in self.clients.values():
            c.close()


class DistributeTranspiler:
    def __init__(self, config=None):
        self.config = config or DistributeTranspilerConfig()
        self._session = None

    # ------------------------------------------------------------------------------ transpile
    def transpile(self, trainer_id, program=None, pservers="127.0.0.1:6174", trainers=1, sync_mode=True,
                  startup_program=None, current_endpoint="127.0.0.1:6174"):
        from ...static import program as P
        from ...static.backward import OPTIMIZE
        self.trainer_id = int(trainer_id)
        self.origin_program = program or P.default_main_program()
        self.origin_startup_program = startup_program or P.default_startup_program()
        self.sync_mode = bool(sync_mode and self.config.sync_mode)
        self.current_endpoint = current_endpoint
        if self.config.mode in ("nccl2", "collective"):
            self.trainers = trainers if isinstance(trainers, int) else len(trainers.split(","))
            return self._transpile_collective()
        if self.config.mode != "pserver":
            raise ValueError(f"DistributeTranspilerConfig.mode must be pserver / nccl2 / collective, got "
                             f"{self.config.mode!r}")
        if self.config.geo_sgd_mode:
            raise NotImplementedError("geo-SGD transpiling: use fleet with a_sync_configs={'k_steps': k} "
                                      "(parallel/ps PSOptimizer geo mode)")
        self.trainers = int(trainers)
        self.pserver_endpoints = [e for e in (pservers.split(",") if isinstance(pservers, str) else pservers) if e]
        blk = self.origin_program.global_block()
        opt_ops = [op for op in blk.ops if op.attrs.get("op_role") == OPTIMIZE and "params" in op.kwargs]
        if len(opt_ops) != 1:
            raise ValueError(f"transpile expects one optimizer op in the program (minimize), found {len(opt_ops)}")
        self._opt_op = opt_ops[0]
        optimizer = self._opt_op.attrs.get("optimizer")
        kind = type(optimizer).__name__.lower() if optimizer is not None else self._opt_op.type
        kind = kind[:-len("optimizer")] if kind.endswith("optimizer") else kind   # fluid's AdamOptimizer ...
        if kind not in _RULES:
            raise NotImplementedError(f"pserver optimizer {kind!r}: the table server implements SGD, Adam and "
                                      f"Adagrad")
        self.rule = _RULES[kind]
        self.lr = float(optimizer.get_lr()) if optimizer is not None else 0.01
        self.rule_kw = {}
        if self.rule == "adam":
            self.rule_kw = dict(beta1=float(getattr(optimizer, "_beta1", 0.9)),
                                beta2=float(getattr(optimizer, "_beta2", 0.999)),
                                epsilon=float(getattr(optimizer, "_epsilon", 1e-8)))
        elif self.rule == "adagrad":
            self.rule_kw = dict(epsilon=float(getattr(optimizer, "_epsilon", 1e-6)),
                                initial_g2sum=float(getattr(optimizer, "initial_accumulator_value", 0.0) or 0.0))
        self.params = list(self._opt_op.kwargs["params"])
        self.grads = list(self._opt_op.kwargs["grads"])
        # ---- blocks and their placement
        n_slices = len(self.pserver_endpoints) if self.config.slice_var_up else 1
        self.blocks = []
        self.by_param = {}
        for p in self.params:
            bl = slice_variable(p, n_slices, self.config.min_block_size)
            self.by_param[p.name] = bl
            self.blocks.extend(bl)
        disp = (self.config.split_method or RoundRobin)(self.pserver_endpoints)
        for b, ep in zip(self.blocks, disp.dispatch(self.blocks)):
            b.endpoint = ep
        for i, b in enumerate(self.blocks):
            b.table = i
        self.param_grad_ep_mapping = {ep: {"params": [b for b in self.blocks if b.endpoint == ep],
                                           "grads": [b for b in self.blocks if b.endpoint == ep]}
                                      for ep in self.pserver_endpoints}
        self._session = _TrainerSession(self)
        self._trainer_program = self._build_trainer_program()

    def _build_trainer_program(self):
        from ...static import program as P
        prog = self.origin_program.clone()
        blk = prog.global_block()
        idx = next(i for i, op in enumerate(blk.ops) if op.fn is self._opt_op.fn)
        del blk.ops[idx]
        sess = self._session
        new_ops = []

        def _send(param, grad, _s=sess):
            _s.send(param, grad)

        def _send_barrier(_s=sess):
            _s.step += 1

        def _recv(param, _s=sess):
            _s.recv(param)

        def _fetch_barrier(_s=sess):
            return None

        ep_of = lambda p: [b.endpoint for b in self.by_param[p.name]]   # noqa: E731
        for p, g in zip(self.params, self.grads):
            new_ops.append(P.OpDesc("send", _send, (), {"param": p, "grad": g}, None, attrs={
                "op_role": "optimize", "epmap": ep_of(p), "sections": [b.row1 - b.row0 for b in self.by_param[p.name]],
                "send_varnames": [b.name for b in self.by_param[p.name]], "sync_mode": self.sync_mode}))
        new_ops.append(P.OpDesc("send_barrier", _send_barrier, (), {}, None,
                                attrs={"op_role": "optimize", "endpoints": list(self.pserver_endpoints),
                                       "trainer_id": self.trainer_id, "half_async": not self.sync_mode}))
        for p in self.params:
            new_ops.append(P.OpDesc("recv", _recv, (), {"param": p}, None, attrs={
                "op_role": "optimize", "epmap": ep_of(p), "recv_varnames": [b.name for b in self.by_param[p.name]],
                "trainer_id": self.trainer_id}))
        new_ops.append(P.OpDesc("fetch_barrier", _fetch_barrier, (), {}, None,
                                attrs={"op_role": "optimize", "endpoints": list(self.pserver_endpoints),
                                       "trainer_id": self.trainer_id}))
        blk.ops[idx:idx] = new_ops
        prog._ps_session = sess
        P.register_close_hook(sess.close)

        # trainer startup: after the local initialisers, trainer 0 creates the server tables from
        # its values and every trainer pulls them (the reference appends recv + fetch_barrier to
        # the trainer's startup program)
        def _init_from_servers(_s=sess):
            if _s.clients is None:
                _s._connect()

        self.origin_startup_program.global_block().append_op(P.OpDesc(
            "recv", _init_from_servers, (), {}, None,
            attrs={"op_role": "optimize", "epmap": list(self.pserver_endpoints), "trainer_id": self.trainer_id}))
        return prog

    def _transpile_collective(self):
        """nccl2 / collective mode: coalesced gradient all-reduce (mean) in front of the optimizer op,
        parameter broadcast from trainer 0 appended to the startup program"""
        from ...static import program as P
        from ...static.backward import OPTIMIZE
        from ...parallel.fleet import static_optimizers as SO
        blk = self.origin_program.global_block()
        for i, op in enumerate(list(blk.ops)):
            if op.attrs.get("op_role") != OPTIMIZE or "grads" not in op.kwargs:
                continue
            grads = tuple(op.kwargs["grads"])
            outs = tuple(P.Variable(blk, g._t, g.name + "@ALLREDUCE") for g in grads)
            for v in outs:
                blk.vars[v.name] = v
            ar = P.OpDesc("c_allreduce_coalesced", SO.c_allreduce_coalesced, (),
                          {"xs": grads, "ring_id": 0, "scale": 1.0 / max(1, self.trainers)}, outs)
            blk.ops.insert(blk.ops.index(op), ar)
            op.kwargs = dict(op.kwargs, grads=outs)
            params = tuple(op.kwargs["params"])
            sb = self.origin_startup_program.global_block()
            sb.ops.append(P.OpDesc("c_broadcast_coalesced", SO.c_broadcast_coalesced, (),
                                   {"xs": params, "root": 0, "ring_id": 0}, None))
        self._trainer_program = self.origin_program
        return None

    # ------------------------------------------------------------------------------ programs
    def get_trainer_program(self, wait_port=True):
        return self._trainer_program

    def get_pserver_program(self, endpoint):
        """one ``listen_and_serv`` op serving ``endpoint``'s blocks until the trainers close"""
        from ...static import program as P
        if self.config.mode != "pserver":
            raise ValueError("get_pserver_program: transpiled in collective mode (no servers)")
        if endpoint not in self.pserver_endpoints:
            raise ValueError(f"{endpoint} is not one of the pserver endpoints {self.pserver_endpoints}")
        prog = P.Program()
        blk = prog.global_block()
        mine = self.param_grad_ep_mapping[endpoint]["params"]
        for b in mine:   # the block variables this server holds (names as the reference's)
            v = P.Variable(blk, torch.empty(b.numel, device="meta"), b.name, persistable=True)
            blk.vars[b.name] = v
        host, port = endpoint.rsplit(":", 1)

        def _listen_and_serv(_port=int(port)):
            from ...parallel.ps import PSServer
            srv = PSServer("0.0.0.0", _port)
            try:
                srv.run()
            finally:
                srv.stop()

        blk.append_op(P.OpDesc("listen_and_serv", _listen_and_serv, (), {}, None, attrs={
            "endpoint": endpoint, "Fanin": self.trainers, "sync_mode": self.sync_mode,
            "pserver_id": self.pserver_endpoints.index(endpoint), "optimize_blocks": [b.name for b in mine],
            "rule": self.rule, "lr": self.lr}))
        return prog

    def get_pserver_programs(self, endpoint):
        main = self.get_pserver_program(endpoint)
        return main, self.get_startup_program(endpoint, main)

    def get_startup_program(self, endpoint, pserver_program=None, startup_program=None):
        """the server's tables are created (with trainer 0's initial values) on the first trainer
        step, so a pserver startup program has nothing to run"""
        from ...static import program as P
        return P.Program()
