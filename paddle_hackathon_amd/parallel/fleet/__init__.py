"""``paddle.distributed.fleet`` (reference: python/paddle/distributed/fleet/base/fleet_base.py,
meta_parallel/{tensor_parallel,pipeline_parallel,sharding_parallel}.py,
meta_optimizers/dygraph_optimizer/hybrid_parallel_optimizer.py).

Collective mode: ``fleet.init`` builds the dp×pp×sharding×mp topology, ``distributed_model``
picks the wrapper, ``distributed_optimizer`` returns a HybridParallelOptimizer (TP/PP-aware
global-norm clip, sharding stage-1). Parameter-server mode (``is_collective=False`` with the
reference's TRAINING_ROLE / PADDLE_PSERVERS_IP_PORT_LIST environment or a UserDefinedRoleMaker):
``init_server``/``run_server`` host the native tables (``parallel/ps``), trainers
``init_worker``, train with ``DistributedEmbedding`` + ``distributed_optimizer`` (PSOptimizer:
sync / async / geo by ``strategy.a_sync`` and ``a_sync_configs["k_steps"]``) and ``stop_worker``.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ...framework.core import Tensor, _wrap
from .. import collective as C
from ..strategy import DistributedStrategy
from ..topology import CommunicateTopology, HybridCommunicateGroup, ParallelMode
from .. import mp_layers, pipeline
from ..data_parallel import DataParallel, sync_params_buffers
from . import meta_parallel, utils  # noqa: F401
from .utils import HybridParallelInferenceHelper  # noqa: F401
from .role_maker import PaddleCloudRoleMaker, UserDefinedRoleMaker, Role  # noqa: F401

__all__ = ["CommunicateTopology", "DistributedStrategy", "Fleet", "HybridCommunicateGroup", "HybridParallelInferenceHelper", "MultiSlotDataGenerator",
           "MultiSlotStringDataGenerator", "PaddleCloudRoleMaker", "Role", "UserDefinedRoleMaker", "UtilBase",
           "init", "distributed_model", "distributed_optimizer", "get_hybrid_communicate_group", "worker_index",
           "worker_num", "is_first_worker", "worker_endpoints", "barrier_worker", "meta_parallel", "utils"]


class UtilBase:
    def all_reduce(self, input, mode="sum", comm_world="worker"):
        import numpy as np
        t = torch.as_tensor(np.asarray(input))
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() and C.get_backend() == "nccl" else torch.device("cpu")
        t = t.to(dev)
        op = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[mode]
        if C.is_initialized():
            dist.all_reduce(t, op=op)
        return t.cpu().numpy()

    def barrier(self, comm_world="worker"):
        C.barrier()

    def all_gather(self, input, comm_world="worker"):
        out = []
        if C.is_initialized():
            C.all_gather_object(out, input)
        else:
            out = [input]
        return out

    def get_file_shard(self, files):
        n, r = worker_num(), worker_index()
        per, extra = divmod(len(files), n)
        start = r * per + min(r, extra)
        return files[start:start + per + (1 if r < extra else 0)]

    def print_on_rank(self, message, rank_id):
        if worker_index() == rank_id:
            print(message)


class Fleet:
    def __init__(self):
        self._hcg = None
        self._strategy = None
        self._role_maker = None
        self._is_collective = True
        self._topology = None
        self._ps = None
        self._dp_model = None
        self.util = UtilBase()
        from . import meta_optimizers as _mo
        _mo._dp_model_hook[0] = lambda: self._dp_model

    def init(self, role_maker=None, is_collective=False, strategy=None, log_level="INFO"):
        self._role_maker = role_maker
        self._strategy = strategy if strategy is not None else DistributedStrategy()
        rm = role_maker if role_maker is not None else PaddleCloudRoleMaker(is_collective=is_collective)
        if not is_collective and rm._is_ps_mode():
            from .. import ps
            self._is_collective = False
            self._role_maker = rm
            self._ps = ps.TheOnePSRuntime(rm, self._strategy)
            ps.set_runtime(self._ps)
            return self
        self._is_collective = True
        self._ps = None
        if not C.is_initialized() and int(os.environ.get("WORLD_SIZE", os.environ.get("PADDLE_TRAINERS_NUM", "1"))) > 1:
            C.init_parallel_env()
        ws = C.get_world_size()
        hc = dict(self._strategy.hybrid_configs)
        mp = max(1, int(hc.get("mp_degree", 1)))
        if mp == 1 and getattr(self._strategy, "tensor_parallel", False):
            # static-graph tensor parallelism (reference tensor_parallel_optimizer.py): the model
            # groups are tensor_parallel_degree consecutive ranks, data parallel across them
            mp = max(1, int((self._strategy.tensor_parallel_configs or {}).get("tensor_parallel_degree", 1)))
        pp = max(1, int(hc.get("pp_degree", 1)))
        sh = max(1, int(hc.get("sharding_degree", 1)))
        dp = int(hc.get("dp_degree", -1))
        if dp <= 0:
            dp = max(1, ws // (mp * pp * sh))
        if dp * mp * pp * sh != ws:
            raise ValueError(f"dp({dp})*mp({mp})*pp({pp})*sharding({sh}) != world size {ws}")
        self._topology = CommunicateTopology(["data", "pipe", "sharding", "model"], [dp, pp, sh, mp])
        self._hcg = HybridCommunicateGroup(self._topology)
        if mp > 1:
            seed = self._strategy.tensor_parallel_configs.get("tensor_init_seed", -1)
            mp_layers.model_parallel_random_seed(None if seed in (-1, None) else seed)
        return self

    # -- role info --------------------------------------------------------------------
    def _ps_mode(self):
        return getattr(self, "_ps", None) is not None

    def worker_index(self):
        return self._role_maker._worker_index() if self._ps_mode() else C.get_rank()

    def worker_num(self):
        return self._role_maker._worker_num() if self._ps_mode() else C.get_world_size()

    def is_first_worker(self):
        return self.is_worker() and self.worker_index() == 0

    def worker_endpoints(self, to_string=False):
        eps = os.environ.get("PADDLE_TRAINER_ENDPOINTS", "")
        lst = eps.split(",") if eps else [f"127.0.0.1:{6170 + i}" for i in range(self.worker_num())]
        return ",".join(lst) if to_string else lst

    def server_num(self):
        return self._role_maker._server_num() if self._ps_mode() else 0

    def server_index(self):
        return self._role_maker._server_index() if self._ps_mode() else 0

    def server_endpoints(self, to_string=False):
        lst = self._role_maker._get_pserver_endpoints() if self._ps_mode() else []
        return ",".join(lst) if to_string else lst

    def is_worker(self):
        return self._role_maker._is_worker() if self._ps_mode() else True

    def is_server(self):
        return self._role_maker._is_server() if self._ps_mode() else False

    def barrier_worker(self):
        if self._ps_mode():
            self._ps.barrier_worker()
        else:
            C.barrier()

    def init_worker(self, scopes=None):
        if self._ps_mode():
            self._ps.init_worker(scopes)

    def init_server(self, *args, **kwargs):
        if self._ps_mode():
            self._ps.init_server(*args, **kwargs)

    def run_server(self):
        if not self._ps_mode():
            raise RuntimeError("run_server() needs parameter-server mode (fleet.init(is_collective=False) with "
                               "TRAINING_ROLE=PSERVER and PADDLE_PSERVERS_IP_PORT_LIST)")
        self._ps.run_server()

    def stop_worker(self):
        if self._ps_mode():
            self._ps.stop_worker()

    def shrink(self, threshold=None):
        """Drop sparse rows unseen for ``threshold`` shrink passes (parameter-server mode)."""
        if self._ps_mode() and self._ps.client is not None:
            for t in sorted(self._ps.client._sparse):
                self._ps.client.shrink(t, int(threshold or 0))

    def get_hybrid_communicate_group(self):
        return self._hcg

    # -- wrappers -------------------------------------------------------------------------
    def distributed_model(self, model):
        if self._ps_mode():
            return model   # dense sync happens in the PS optimizer, sparse tables in DistributedEmbedding
        hcg, st = self._hcg, self._strategy
        if hcg is None:
            self.init(is_collective=True)
            hcg, st = self._hcg, self._strategy
        mode = hcg.get_parallel_mode()
        if mode == ParallelMode.PIPELINE_PARALLEL:
            return pipeline.PipelineParallel(model, hcg, st)
        if mode == ParallelMode.TENSOR_PARALLEL:
            return TensorParallel(model, hcg, st)
        if mode == ParallelMode.SHARDING_PARALLEL:
            return ShardingParallel(model, hcg, st)
        if C.get_world_size() > 1:
            self._dp_model = DataParallel(model, comm_buffer_size=st.fuse_grad_size_in_MB,
                                          last_comm_buffer_size=st.last_comm_group_size_MB,
                                          find_unused_parameters=st.find_unused_parameters,
                                          group=hcg.get_data_parallel_group())
            if st.fp16_allreduce and self._dp_model._reducer is not None:
                self._dp_model._reducer.comm_dtype = torch.bfloat16
            return self._dp_model
        return model

    def distributed_optimizer(self, optimizer, strategy=None):
        if strategy is not None:
            self._strategy = strategy
        if self._ps_mode():
            from ..ps import PSOptimizer
            self._ps.strategy = self._strategy
            return PSOptimizer(optimizer, self._ps, self._strategy)
        if not _core_in_dynamic():
            # static graph: meta-optimizers rewrite the Program (static_optimizers.py); pipeline
            # parallelism runs the stage program of this rank (static_pipeline.py)
            st = self._strategy
            if st is not None and getattr(st, "pipeline", False):
                from .static_pipeline import PipelineOptimizer
                cfg = dict(getattr(st, "pipeline_configs", {}) or {})
                return PipelineOptimizer(optimizer, int(cfg.get("accumulate_steps", 1)))
            from .static_optimizers import StaticFleetOptimizer
            return StaticFleetOptimizer(optimizer, self._strategy)
        if self._hcg is None:
            self.init(is_collective=True)
        from . import meta_optimizers as mo
        optimizer = mo.apply_meta_optimizers(optimizer, self._strategy, self._dp_model)
        hp = HybridParallelOptimizer(optimizer, self._hcg, self._strategy)
        dp_g = self._hcg.get_data_parallel_group() if self._hcg is not None else None
        return mo.wrap_meta_optimizers(hp, self._strategy, self._dp_model, group=dp_g if dp_g is not None and dp_g.nranks > 1 else None)

    def distributed_scaler(self, scaler):
        return scaler

    # -- persistence ------------------------------------------------------------------------
    def save_persistables(self, executor=None, dirname=None, main_program=None, mode=0):
        """Parameter-server mode: every table of the job (dense and sparse) into ``dirname``,
        one file per table per server (mode 0 with optimizer state, 1 weights only)."""
        if self._ps_mode() and self._ps.client is not None and dirname:
            c = self._ps.client
            for t in sorted(set(c._dense) | set(c._sparse)):
                c.save(t, dirname, mode)

    def load_persistables(self, dirname):
        if self._ps_mode() and self._ps.client is not None:
            c = self._ps.client
            for t in sorted(set(c._dense) | set(c._sparse)):
                c.load(t, dirname)

    def save_inference_model(self, *args, **kwargs):
        from ...static import save_inference_model
        return save_inference_model(*args, **kwargs)

    def state_dict(self):
        return {}


class TensorParallel:
    """Wraps a TP model: broadcast non-distributed params inside the mp group (and everything
    inside the dp group), and data-parallel reduce over the dp group."""

    def __new__(cls, model, hcg, strategy):
        mp_g = hcg.get_model_parallel_group()
        if mp_g is not None and mp_g.nranks > 1:
            sync_params_buffers(model, mp_g, 0, is_model_parallel=True)
        dp_g = hcg.get_data_parallel_group()
        if dp_g is not None and dp_g.nranks > 1:
            return DataParallel(model, comm_buffer_size=strategy.fuse_grad_size_in_MB,
                                last_comm_buffer_size=strategy.last_comm_group_size_MB, group=dp_g)
        return model


class ShardingParallel:
    def __new__(cls, model, hcg, strategy):
        g = hcg.get_sharding_parallel_group()
        if g is not None and g.nranks > 1:
            sync_params_buffers(model, g, 0)
        return model


class HybridParallelOptimizer:
    """TP/PP/sharding-aware optimizer wrapper (reference: hybrid_parallel_optimizer.py)."""

    def __init__(self, optimizer, hcg, strategy):
        self._inner_opt = optimizer
        self._hcg = hcg
        self._strategy = strategy
        mode = hcg.get_parallel_mode() if hcg is not None else ParallelMode.DATA_PARALLEL
        clip = optimizer._grad_clip
        from ...nn.clip import ClipGradByGlobalNorm
        if isinstance(clip, ClipGradByGlobalNorm) and hcg is not None:
            cg = hcg.get_check_parallel_group()
            if cg is not None and cg.nranks > 1 and cg.pg is not None:
                clip._check_group = cg.pg
                clip._mp_degree = hcg.get_model_parallel_world_size()
                plist = optimizer._parameter_list or []
                clip._device = plist[0]._t.device if plist else None
        self._sharding = None
        sg = hcg.get_sharding_parallel_group() if hcg is not None else None
        if sg is not None and sg.nranks > 1:
            from ..sharding import ShardingOptimizerStage1
            self._sharding = ShardingOptimizerStage1(optimizer, sg, hcg.get_data_parallel_group())

    def step(self):
        if self._sharding is not None:
            return self._sharding.step()
        return self._inner_opt.step()

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        self.step()

    def clear_grad(self, set_to_zero=True):
        if self._sharding is not None:
            return self._sharding.clear_grad(set_to_zero)
        self._inner_opt.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def __getattr__(self, item):
        return getattr(self._inner_opt, item)


fleet = Fleet()
init = fleet.init
distributed_model = fleet.distributed_model
distributed_optimizer = fleet.distributed_optimizer
distributed_scaler = fleet.distributed_scaler
get_hybrid_communicate_group = fleet.get_hybrid_communicate_group
worker_index = fleet.worker_index
worker_num = fleet.worker_num
is_first_worker = fleet.is_first_worker
worker_endpoints = fleet.worker_endpoints
server_num = fleet.server_num
is_worker = fleet.is_worker
is_server = fleet.is_server
barrier_worker = fleet.barrier_worker
init_worker = fleet.init_worker
init_server = fleet.init_server
run_server = fleet.run_server
stop_worker = fleet.stop_worker
save_persistables = fleet.save_persistables
load_persistables = fleet.load_persistables
shrink = fleet.shrink
server_index = fleet.server_index
server_endpoints = fleet.server_endpoints
save_inference_model = fleet.save_inference_model
util = fleet.util


class MultiSlotDataGenerator:
    """Slot-format sample generator (reference: fleet/data_generator/data_generator.py)."""

    def set_batch(self, batch_size):
        self.batch_size_ = batch_size

    def generate_sample(self, line):
        raise NotImplementedError

    def generate_batch(self, samples):
        def gen():
            for s in samples:
                yield s
        return gen

    def _format(self, sample):
        out = []
        for name, vals in sample:
            out.append(str(len(vals)))
            out.extend(str(v) for v in vals)
        return " ".join(out)

    def run_from_memory(self, lines):
        res = []
        for line in lines:
            for s in self.generate_sample(line)():
                res.append(self._format(s))
        return res

    def run_from_stdin(self):
        import sys
        for line in sys.stdin:
            for s in self.generate_sample(line)():
                sys.stdout.write(self._format(s) + "\n")


class MultiSlotStringDataGenerator(MultiSlotDataGenerator):
    pass


def __getattr__(name):   # submodules imported lazily (fleet.elastic is also a `python -m` entry point)
    import importlib
    if name in ("elastic", "metrics", "data_generator", "base", "runtime", "recompute"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)


def _core_in_dynamic():
    from ...framework import core
    return core.in_dynamic_mode()
