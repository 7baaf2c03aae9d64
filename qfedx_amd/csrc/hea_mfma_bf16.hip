// bf16 build of the MFMA statevector engine (BASELINE config 2: "16-qubit VQC FedAvg bf16"): the kernels of
// hea_mfma.hip with bf16 (re, im) state storage, bf16 hi + lo unitary fragments and v_mfma_f32_16x16x32_bf16, in
// namespace hea_bf16 with _bf16 entry points.  fp32 accumulation and the 2^(n/2) state scale are unchanged (bf16 has
// fp32's exponent range, so the scale is harmless); the per-op rounding of the state is 2^-9 instead of 2^-12.
#define QFX_HEA_BF16 1
#include "hea_mfma.hip"
#include "hea_step.hip"
