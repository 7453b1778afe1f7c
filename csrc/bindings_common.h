// Shared helpers for the torch-facing binding translation units.
#pragma once
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>

#define FAN_T_CUDA_CONTIG(t)                                                       \
  TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor");                         \
  TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")

inline hipStream_t fan_stream() { return c10::hip::getCurrentHIPStream().stream(); }
