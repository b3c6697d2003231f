"""Analytic cost estimate of a sharded training step (reference:
python/paddle/distributed/auto_parallel/cost_model.py: estimate_cost over a distributed Program,
cluster model and per-op standalone costs).

Here the inputs are a model (or a parameter list) and the per-parameter ``dims_mapping``
annotations on a :class:`ProcessMesh`; the estimate prices the compute at the MI355X bf16 MFMA rate and
the gradient / activation collectives as ring collectives over xGMI (7 point-to-point links of
≈153 GB/s per GPU), so it can rank sharding plans before anything runs."""
from __future__ import annotations

import numpy as np

__all__ = ["estimate_cost", "MI355X"]

MI355X = {"bf16_flops": 2.5e15, "mfma_efficiency": 0.55, "hbm_bw": 8e12, "xgmi_link_bw": 153e9, "xgmi_links": 7,
          "collective_latency": 20e-6}


def _ring(bytes_, n, bw, lat):
    """Ring all-reduce time of ``bytes_`` over ``n`` ranks at per-rank bandwidth ``bw``."""
    if n <= 1 or bytes_ <= 0:
        return 0.0
    return 2.0 * (n - 1) / n * bytes_ / bw + 2 * (n - 1) * lat


def estimate_cost(distributed_program=None, cluster=None, pipeline_config=None, standalone_cost_data=None,
                  batch_size=1, tokens_per_sample=1, process_mesh=None, dtype_bytes=2):
    """Estimated seconds per training step: ``{"compute", "grad_allreduce", "param_comm", "total",
    "params", "flops"}``. ``distributed_program``: a Layer, or an iterable of parameters."""
    from .process_mesh import get_default_mesh
    hw = dict(MI355X, **(cluster or {})) if isinstance(cluster, dict) else MI355X
    mesh = process_mesh or get_default_mesh()
    params = list(distributed_program.parameters()) if hasattr(distributed_program, "parameters") \
        else list(distributed_program or [])
    shape = mesh.topology
    n_total = int(np.prod(shape))
    total_params, local_params, grad_bytes, tp_bytes, tp_group = 0, 0.0, 0.0, 0.0, 1
    rows = batch_size * tokens_per_sample
    for p in params:
        shp = [int(d) for d in p.shape]
        numel = int(np.prod(shp))
        total_params += numel
        dm = (getattr(p, "dist_attr", None) or {}).get("dims_mapping") or [-1] * len(shp)
        split = int(np.prod([shape[m] for m in dm if m >= 0])) if any(m >= 0 for m in dm) else 1
        local_params += numel / split
        # gradients are summed over the mesh dims the parameter is replicated on (data parallel)
        if n_total // split > 1:
            grad_bytes += numel / split * dtype_bytes
        # Megatron pairs: a row-split [in, out] weight all-reduces its [rows, out] output (fwd);
        # a column-split one all-reduces its [rows, in] input gradient (bwd)
        if len(shp) == 2 and split > 1:
            tp_group = max(tp_group, split)
            tp_bytes += rows * (shp[1] if dm[0] >= 0 else shp[0]) * dtype_bytes
    flops = 6.0 * local_params * rows
    compute = flops / (hw["bf16_flops"] * hw["mfma_efficiency"])
    link_bw = hw["xgmi_link_bw"] * hw["xgmi_links"] / 2      # ring: both directions share the links
    dp_size = max(1, n_total // tp_group)
    grad = _ring(grad_bytes, dp_size, link_bw, hw["collective_latency"])
    act = _ring(tp_bytes, tp_group, link_bw, hw["collective_latency"])
    # bucketed gradient all-reduce overlaps backward (~2/3 of the compute); TP collectives do not
    exposed_grad = max(0.0, grad - compute * 2.0 / 3.0)
    return {"compute": compute, "grad_allreduce": grad, "param_comm": act, "total": compute + exposed_grad + act,
            "params": total_params, "flops": flops}
