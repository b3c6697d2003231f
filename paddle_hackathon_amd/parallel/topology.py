"""Hybrid-parallel topology (reference: python/paddle/distributed/fleet/base/topology.py).

Axis order is ["data", "pipe", "sharding", "model"] with the model (tensor-parallel)
axis fastest-varying, so a TP group is a run of consecutive ranks = GPUs of one
node joined by xGMI; DP/sharding groups stride across them.
"""
from __future__ import annotations

import collections
import itertools
from functools import reduce

import numpy as np

from . import collective as C

__all__ = ["CommunicateTopology", "HybridCommunicateGroup", "ParallelMode"]


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3


class CommunicateTopology:
    def __init__(self, hybrid_group_names=("data", "pipe", "sharding", "model"), dims=(1, 1, 1, 1)):
        self._parallel_names = list(hybrid_group_names)
        self._dims = list(dims)
        self.coordinate = collections.namedtuple("Coordinate", self._parallel_names)
        self._world_size = reduce(lambda a, b: a * b, self._dims, 1)
        ranges = [range(d) for d in self._dims]
        all_coords = [self.coordinate(*x) for x in itertools.product(*ranges)]
        self._coord2rank = dict(zip(all_coords, range(len(all_coords))))
        self._rank2coord = dict(zip(self._coord2rank.values(), self._coord2rank.keys()))

    def get_hybrid_group_names(self):
        return self._parallel_names

    def get_dim(self, axis_name):
        return self._dims[self._parallel_names.index(axis_name)]

    def world_size(self):
        return self._world_size

    def get_rank(self, **args):
        return self._coord2rank[self.coordinate(**args)]

    def get_coord(self, rank):
        return self._rank2coord[rank]

    def get_axis_list(self, axis_name, index):
        axis = self._parallel_names.index(axis_name)
        return sorted(r for c, r in self._coord2rank.items() if c[axis] == index)

    def get_dim_size(self, axis_name):
        return self.get_dim(axis_name)

    def get_comm_list(self, axis_name):
        """All groups along ``axis_name``: lists of ranks that differ only in that coordinate."""
        axis = self._parallel_names.index(axis_name)
        others = [range(d) for i, d in enumerate(self._dims) if i != axis]
        out = []
        for o in itertools.product(*others):
            grp = []
            for k in range(self._dims[axis]):
                coord = list(o)
                coord.insert(axis, k)
                grp.append(self._coord2rank[self.coordinate(*coord)])
            out.append(grp)
        return out

    def get_rank_from_stage(self, global_rank, **kwargs):
        coord = self.get_coord(global_rank)._asdict()
        coord.update(kwargs)
        return self.get_rank(**coord)


class HybridCommunicateGroup:
    def __init__(self, topology):
        self._topo = topology
        self.global_rank = C.get_rank()
        self.nranks = topology.world_size()
        self._dp_degree = topology.get_dim("data")
        self._mp_degree = topology.get_dim("model")
        self._pp_degree = topology.get_dim("pipe")
        self._sharding_degree = topology.get_dim("sharding")
        self._data_parallel_id = self._get_id("data")
        self._model_parallel_id = self._get_id("model")
        self._sharding_parallel_id = self._get_id("sharding")
        self.stage_id = self._get_id("pipe")
        self._dp_group, self._dp_comm_group = self._set_comm_group("data")
        self._mp_group, self._mp_comm_group = self._set_comm_group("model")
        self._pp_group, self._pp_comm_group = self._set_comm_group("pipe")
        self._sharding_group, self._sharding_comm_group = self._set_comm_group("sharding")
        # "check" group = everything but data parallel (for global-norm clip / found_inf)
        self._check_group, self._check_comm_group = self._set_check_group()
        self.is_first_stage = self.stage_id == 0
        self.is_last_stage = self.stage_id == self._pp_degree - 1
        self._p2p_next = self._topo.get_rank_from_stage(self.global_rank, pipe=(self.stage_id + 1) % self._pp_degree)
        self._p2p_prev = self._topo.get_rank_from_stage(self.global_rank, pipe=(self.stage_id - 1) % self._pp_degree)

    def _get_id(self, axis):
        return getattr(self._topo.get_coord(self.global_rank), axis)

    def _set_comm_group(self, axis):
        my_ranks, my_group = None, None
        for ranks in self._topo.get_comm_list(axis):
            g = C.new_group(ranks) if C.is_initialized() and len(ranks) > 1 else None
            if self.global_rank in ranks:
                my_ranks = ranks
                my_group = g if g is not None else C.Group(ranks.index(self.global_rank), -1, ranks, None)
        return my_ranks, my_group

    def _set_check_group(self):
        axis = "data"
        idx = self._topo._parallel_names.index(axis)
        groups = collections.defaultdict(list)
        for r in range(self.nranks):
            c = self._topo.get_coord(r)
            groups[c[idx]].append(r)
        my_ranks, my_group = None, None
        for key in sorted(groups):
            ranks = groups[key]
            g = C.new_group(ranks) if C.is_initialized() and len(ranks) > 1 else None
            if self.global_rank in ranks:
                my_ranks = ranks
                my_group = g if g is not None else C.Group(ranks.index(self.global_rank), -1, ranks, None)
        return my_ranks, my_group

    def get_parallel_mode(self):
        if self._mp_degree == 1 and self._pp_degree == 1 and self._sharding_degree == 1:
            return ParallelMode.DATA_PARALLEL
        if self._mp_degree > 1 and self._pp_degree == 1:
            return ParallelMode.TENSOR_PARALLEL
        if self._pp_degree > 1:
            return ParallelMode.PIPELINE_PARALLEL
        return ParallelMode.SHARDING_PARALLEL

    def topology(self):
        return self._topo

    def get_global_rank(self):
        return self.global_rank

    # data parallel
    def get_data_parallel_rank(self):
        return self._data_parallel_id

    def get_data_parallel_world_size(self):
        return self._dp_degree

    def get_data_parallel_group(self):
        return self._dp_comm_group

    def get_data_parallel_group_src_rank(self):
        return self._dp_group[0]

    # model (tensor) parallel
    def get_model_parallel_rank(self):
        return self._model_parallel_id

    def get_model_parallel_world_size(self):
        return self._mp_degree

    def get_model_parallel_group(self):
        return self._mp_comm_group

    def get_model_parallel_group_src_rank(self):
        return self._mp_group[0]

    # pipeline
    def get_stage_id(self):
        return self.stage_id

    def get_pipe_parallel_world_size(self):
        return self._pp_degree

    def get_pipe_parallel_group(self):
        return self._pp_comm_group

    def get_p2p_groups(self):
        return None

    # sharding
    def get_sharding_parallel_rank(self):
        return self._sharding_parallel_id

    def get_sharding_parallel_world_size(self):
        return self._sharding_degree

    def get_sharding_parallel_group(self):
        return self._sharding_comm_group

    def get_sharding_parallel_group_src_rank(self):
        return self._sharding_group[0]

    def get_check_parallel_group(self):
        return self._check_comm_group

    def get_rank_from_stage(self, stage_id, **kwargs):
        return self._topo.get_rank_from_stage(self.global_rank, pipe=stage_id, **kwargs)
