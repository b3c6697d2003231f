// A C++ service-style client of libpha_infer.so through the reference's C API subset (PD_Config /
// PD_Predictor / PD_Tensor, as in paddle/fluid/inference/capi_exp): loads a saved model, feeds
// inputs read from raw files, runs, and writes every output to <out_prefix><i>.bin with its shape
// on stdout. tests/test_native_infer.py builds it with g++ and compares against the Python
// predictor.
//
//   infer_main MODEL PARAMS DEVICE OUT_PREFIX NAME:DTYPE:D0,D1,...:FILE [...]
//   DTYPE: f32 | i64 ; DEVICE: -1 host, k >= 0 GPU k
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "pha_infer.h"

static std::vector<std::string> split(const std::string& s, char d) {
  std::vector<std::string> r;
  size_t a = 0;
  for (size_t b; (b = s.find(d, a)) != std::string::npos; a = b + 1) r.push_back(s.substr(a, b - a));
  r.push_back(s.substr(a));
  return r;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s MODEL PARAMS DEVICE OUT_PREFIX NAME:DTYPE:DIMS:FILE ...\n", argv[0]);
    return 2;
  }
  const int dev = std::atoi(argv[3]);
  PD_Config* cfg = PD_ConfigCreate();
  PD_ConfigSetModel(cfg, argv[1], argv[2]);
  if (dev >= 0) PD_ConfigEnableUseGpu(cfg, 256, dev);
  else PD_ConfigDisableGpu(cfg);
  PD_Predictor* pred = PD_PredictorCreate(cfg);   // takes the config
  if (!pred) return 3;
  PD_OneDimArrayCstr* in_names = PD_PredictorGetInputNames(pred);
  std::printf("inputs %zu outputs %zu\n", PD_PredictorGetInputNum(pred), PD_PredictorGetOutputNum(pred));
  for (int a = 5; a < argc; ++a) {
    auto f = split(argv[a], ':');
    if (f.size() != 4) return 2;
    std::vector<int32_t> shape;
    size_t n = 1;
    for (auto& d : split(f[2], ',')) {
      shape.push_back(std::atoi(d.c_str()));
      n *= (size_t)shape.back();
    }
    const size_t es = f[1] == "i64" ? 8 : 4;
    std::vector<char> buf(n * es);
    std::ifstream in(f[3], std::ios::binary);
    in.read(buf.data(), (std::streamsize)buf.size());
    if (!in) {
      std::fprintf(stderr, "short input file %s\n", f[3].c_str());
      return 2;
    }
    PD_Tensor* t = PD_PredictorGetInputHandle(pred, f[0].c_str());
    PD_TensorReshape(t, shape.size(), shape.data());
    if (f[1] == "i64") PD_TensorCopyFromCpuInt64(t, reinterpret_cast<const int64_t*>(buf.data()));
    else PD_TensorCopyFromCpuFloat(t, reinterpret_cast<const float*>(buf.data()));
    PD_TensorDestroy(t);
  }
  PD_OneDimArrayCstrDestroy(in_names);
  if (!PD_PredictorRun(pred)) return 4;
  PD_OneDimArrayCstr* out_names = PD_PredictorGetOutputNames(pred);
  for (size_t i = 0; i < out_names->size; ++i) {
    PD_Tensor* t = PD_PredictorGetOutputHandle(pred, out_names->data[i]);
    PD_OneDimArrayInt32* s = PD_TensorGetShape(t);
    size_t n = 1;
    std::printf("output %zu %s shape", i, PD_TensorGetName(t));
    for (size_t k = 0; k < s->size; ++k) {
      std::printf(" %d", s->data[k]);
      n *= (size_t)s->data[k];
    }
    std::printf("\n");
    std::vector<float> out(n);
    PD_TensorCopyToCpuFloat(t, out.data());
    std::ofstream o(std::string(argv[4]) + std::to_string(i) + ".bin", std::ios::binary);
    o.write(reinterpret_cast<const char*>(out.data()), (std::streamsize)(n * sizeof(float)));
    PD_OneDimArrayInt32Destroy(s);
    PD_TensorDestroy(t);
  }
  PD_OneDimArrayCstrDestroy(out_names);
  PD_PredictorDestroy(pred);
  return 0;
}
