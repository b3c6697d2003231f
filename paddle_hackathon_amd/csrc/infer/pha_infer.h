// Native inference API of paddle_hackathon_amd (libpha_infer.so): loads a saved inference model
// (.pdmodel ProgramDesc + .pdiparams save_combine stream, the reference's file formats) and runs
// its block 0 with a C++ graph walker — no Python, no torch. On device >= 0 every op runs on the
// MI355X through the library's own HIP kernels (fp32 MFMA GEMM / implicit-im2col convolution,
// fused elementwise, norm, softmax and pooling kernels); on device -1 the same graph runs on the
// host (reference loops, the numerics oracle of the GPU path).
//
// Two API layers:
//  * pha_infer_*  — a minimal handle API (create / set_input / run / get_output / destroy);
//  * PD_*         — the subset of the reference's C API (paddle/fluid/inference/capi_exp/
//                   pd_config.h, pd_predictor.h, pd_tensor.h) a C / C++ service needs to run a model:
//                   config, predictor, input / output handles, reshape, copy from / to CPU.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---- handle API -------------------------------------------------------------------------------
typedef struct PhaPredictor PhaPredictor;

// element types: the reference's VarType codes
enum { PHA_INT32 = 2, PHA_INT64 = 3, PHA_FLOAT32 = 5 };

// device: -1 = host, k >= 0 = GPU k. NULL on failure (pha_infer_last_error says why).
PhaPredictor* pha_infer_create(const char* model_file, const char* params_file, int device);
const char* pha_infer_last_error(void);
int pha_infer_num_inputs(const PhaPredictor* p);
const char* pha_infer_input_name(const PhaPredictor* p, int i);
int pha_infer_num_outputs(const PhaPredictor* p);
const char* pha_infer_output_name(const PhaPredictor* p, int i);
// copies host data into the named input (0 = ok)
int pha_infer_set_input(PhaPredictor* p, const char* name, int dtype, const int64_t* shape, int ndim,
                        const void* data);
int pha_infer_run(PhaPredictor* p);
// output i's shape (up to 8 dims) and element type
int pha_infer_output_shape(const PhaPredictor* p, int i, int64_t* shape, int* ndim, int* dtype);
// copies output i to host memory of `bytes` bytes
int pha_infer_copy_output(const PhaPredictor* p, int i, void* dst, size_t bytes);
// op types of the loaded program the engine cannot run ("" when none)
const char* pha_infer_unsupported_ops(const PhaPredictor* p);
// ir_optim = 0: run the program as written (no conv + elementwise_add / conv + batch_norm folding)
PhaPredictor* pha_infer_create2(const char* model_file, const char* params_file, int device, int ir_optim);
// bf16 != 0: the GPU path's matrix products run with bf16 operands on libpha_kernels.so's MFMA GEMM
PhaPredictor* pha_infer_create3(const char* model_file, const char* params_file, int device, int ir_optim, int bf16);
// the IR passes that rewrote the program at load ("conv_bn_fuse_pass x53;..."; "" when none)
const char* pha_infer_applied_passes(const PhaPredictor* p);
// device bytes held by the predictor's block pool (0 on the host)
size_t pha_infer_pooled_bytes(const PhaPredictor* p);
void pha_infer_destroy(PhaPredictor* p);

// ---- reference C API subset -------------------------------------------------------------------
typedef int8_t PD_Bool;
typedef struct PD_Config PD_Config;
typedef struct PD_Predictor PD_Predictor;
typedef struct PD_Tensor PD_Tensor;
typedef struct PD_OneDimArrayCstr {
  size_t size;
  char** data;
} PD_OneDimArrayCstr;
typedef struct PD_OneDimArrayInt32 {
  size_t size;
  int32_t* data;
} PD_OneDimArrayInt32;

PD_Config* PD_ConfigCreate(void);
void PD_ConfigSwitchIrOptim(PD_Config* c, PD_Bool x);
PD_Bool PD_ConfigIrOptim(PD_Config* c);
void PD_ConfigEnableMkldnnBfloat16(PD_Config* c);
PD_Bool PD_ConfigMkldnnBfloat16Enabled(PD_Config* c);
void PD_ConfigDestroy(PD_Config* c);
void PD_ConfigSetModel(PD_Config* c, const char* prog_file_path, const char* params_file_path);
const char* PD_ConfigGetProgFile(PD_Config* c);
const char* PD_ConfigGetParamsFile(PD_Config* c);
void PD_ConfigEnableUseGpu(PD_Config* c, uint64_t memory_pool_init_size_mb, int32_t device_id);
void PD_ConfigDisableGpu(PD_Config* c);
PD_Bool PD_ConfigUseGpu(PD_Config* c);
int32_t PD_ConfigGpuDeviceId(PD_Config* c);

// takes ownership of (and destroys) the config, as the reference does
PD_Predictor* PD_PredictorCreate(PD_Config* c);
void PD_PredictorDestroy(PD_Predictor* p);
size_t PD_PredictorGetInputNum(PD_Predictor* p);
size_t PD_PredictorGetOutputNum(PD_Predictor* p);
PD_OneDimArrayCstr* PD_PredictorGetInputNames(PD_Predictor* p);
PD_OneDimArrayCstr* PD_PredictorGetOutputNames(PD_Predictor* p);
PD_Tensor* PD_PredictorGetInputHandle(PD_Predictor* p, const char* name);
PD_Tensor* PD_PredictorGetOutputHandle(PD_Predictor* p, const char* name);
PD_Bool PD_PredictorRun(PD_Predictor* p);
void PD_OneDimArrayCstrDestroy(PD_OneDimArrayCstr* a);
void PD_OneDimArrayInt32Destroy(PD_OneDimArrayInt32* a);

void PD_TensorDestroy(PD_Tensor* t);
void PD_TensorReshape(PD_Tensor* t, size_t shape_size, int32_t* shape);
void PD_TensorCopyFromCpuFloat(PD_Tensor* t, const float* data);
void PD_TensorCopyFromCpuInt64(PD_Tensor* t, const int64_t* data);
void PD_TensorCopyFromCpuInt32(PD_Tensor* t, const int32_t* data);
void PD_TensorCopyToCpuFloat(PD_Tensor* t, float* data);
void PD_TensorCopyToCpuInt64(PD_Tensor* t, int64_t* data);
void PD_TensorCopyToCpuInt32(PD_Tensor* t, int32_t* data);
PD_OneDimArrayInt32* PD_TensorGetShape(PD_Tensor* t);
const char* PD_TensorGetName(PD_Tensor* t);

#ifdef __cplusplus
}
#endif
