"""One kernel-name classifier for every profile summary (tools/trace_window.py,
tools/prof_summary.py): own HIP kernels by family, library kernels by library — so a summary never
files the own GEMMs under a library name or the library GEMMs under "other"."""
import re

# (label, predicate) in priority order
_RULES = [
    ("own GEMM (gemm4p/gemm4w/gemm8p)", lambda n: re.search(r"pha::g4[pw]::|pha::g8p::|gemm4[pw]_kernel|gemm8p_kernel", n)),
    ("own conv GEMM (gemm256/gemm_conv)", lambda n: re.search(r"gemm256|conv256|gemm_conv|conv_gemm|pha::g256::", n)),
    ("own flash attention", lambda n: re.search(r"\bfa_|\bfa64_|flash|attn", n) and "at::native" not in n),
    ("own layer_norm / softmax / CE", lambda n: re.search(r"ln_fwd|ln_bwd|col_reduce|col_partial|softmax|_ce_|bdrln", n)
     and "at::native" not in n),
    ("own batch_norm", lambda n: re.search(r"\bbn_|batch_norm", n) and "MIOpen" not in n and "at::native" not in n),
    ("own optimizer (adam/momentum/l2)", lambda n: re.search(r"adam_kernel|momentum_kernel|l2sq|sum_partials", n)),
    ("own other HIP kernels", lambda n: ("pha::" in n or "anonymous namespace)::" in n) and "at::native" not in n),
    ("LIBRARY hipBLASLt/Tensile GEMM", lambda n: n.startswith("Cijk") or n.startswith("Custom_Cijk")),
    ("LIBRARY MIOpen", lambda n: "miopen" in n.lower() or "MIOpen" in n or n.startswith("naive_conv")
     or "igemm" in n or "BatchNorm" in n),
    ("LIBRARY rocBLAS", lambda n: "rocblas" in n.lower()),
    ("torch native (elementwise/reduce/copy)", lambda n: "at::native" in n),
    ("runtime fills/copies", lambda n: "__amd_rocclr" in n),
    ("RCCL", lambda n: "nccl" in n.lower() or "rccl" in n.lower()),
]


def classify(name):
    for label, pred in _RULES:
        if pred(name):
            return label
    return "other"


def is_library(name):
    return classify(name).startswith("LIBRARY")
