// Gradient bucket planning for data-parallel / sharded all-reduce (reference behaviour:
// paddle/fluid/imperative/reducer.cc AssignGroupBySize and
// python/paddle/fluid/dygraph/parallel.py build_groups).
//
// Parameters are visited in the order their gradients become ready (reverse registration
// order by default). A bucket closes when adding the next tensor would exceed the current
// byte limit; limits are consumed from `limits` (a small first bucket lets the first RCCL
// all-reduce start early in backward; later buckets are large so each ring pass over xGMI
// moves enough bytes to saturate the per-link bandwidth). Different dtypes never share a
// bucket; sparse gradients always get a bucket of their own.
#include <algorithm>
#include <map>
#include <vector>

#include "runtime.h"

PHA_API int pha_plan_buckets(int64_t n, const int64_t* nbytes, const int32_t* dtype_ids, const uint8_t* is_sparse,
                             const int64_t* limits, int nlimits, const int64_t* order, int32_t* out_group) {
  if (n <= 0) return 0;
  if (nlimits <= 0) return -1;
  struct Open {
    int32_t gid;
    int64_t bytes;
    int limit_idx;
  };
  std::map<int32_t, Open> open;  // dtype -> currently filling bucket
  int32_t next_gid = 0;
  int limit_cursor = 0;  // limits are handed out in bucket-creation order across dtypes
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = order ? order[k] : k;
    if (i < 0 || i >= n) return -1;
    if (is_sparse && is_sparse[i]) {
      out_group[i] = next_gid++;
      continue;
    }
    auto it = open.find(dtype_ids[i]);
    if (it != open.end()) {
      Open& b = it->second;
      const int64_t lim = limits[std::min(b.limit_idx, nlimits - 1)];
      if (b.bytes + nbytes[i] <= lim || b.bytes == 0) {
        b.bytes += nbytes[i];
        out_group[i] = b.gid;
        continue;
      }
    }
    Open b{next_gid++, nbytes[i], limit_cursor++};
    out_group[i] = b.gid;
    open[dtype_ids[i]] = b;
  }
  return next_gid;
}

// Elements to pad a flat bucket to so reduce-scatter gives every rank an equal, aligned
// shard (align_elems keeps each shard 16-byte aligned for vectorised HIP kernels).
PHA_API int64_t pha_bucket_padded_numel(int64_t numel, int64_t world, int64_t align_elems) {
  if (world < 1) world = 1;
  if (align_elems < 1) align_elems = 1;
  const int64_t unit = world * align_elems;
  return (numel + unit - 1) / unit * unit;
}
