// Device-resident data path: one padded batch gathered from the feature store in HBM.
//
// Replaces, per batch, the DataLoader's per-sample row-slice copy + .float()
//   NoisyEmotionDatasetFromArrays.__getitem__   I/dataload_noisy.py:104-115
//   CleanEmotionDatasetFromArrays.__getitem__   I/dataload_clean.py:170-176
//   (CASIA/EMODB: C/dataload_casia_noisy.py:49-66)
// and the collator's zero padding + padding mask + label gather
//   collator                                    I/dataload_noisy.py:116-129, I/dataload_clean.py:177-193,
//                                               C/dataload_casia_noisy.py:68-99
// The whole feature set (IEMOCAP ~3.8 GB f32) stays resident in HBM for the run; a batch is a
// list of sample indices, and collation is this gather: no host copy, no H2D per step.
//
// Work: row r of the [B][T] output (b = r / T, t = r % T) is 768 features = 3 KB: one wave per
// row, 3 x 16 B per lane (fully coalesced), rows past the sample's size are written as zeros
// without reading.  HBM-bound byte work: algorithmic bytes per batch = store bytes of the
// valid rows read + 3072 B x B x T written + B x T mask bytes.  Each wave takes kRowsPerWave
// consecutive rows with all their loads issued before the first store (6 loads in flight per
// lane); the store is read once per epoch, so its loads are non-temporal (they do not evict
// the output the encoder reads next from L2).
#include <cstring>

#include "dad_common.h"
#include "dad_kernels.h"

namespace {

constexpr int kWaves = DAD_COLLATE_THREADS / 64;
constexpr int kRowsPerWave = 2;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int DT>
struct StoreRow;

template <>
struct StoreRow<DAD_STORE_F32> {
  f32x4 v[3];
  __device__ __forceinline__ void load(const void* base, long frame, int lane) {
    const f32x4* p = reinterpret_cast<const f32x4*>(base) + (size_t)frame * (DAD_D / 4) + lane;
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = __builtin_nontemporal_load(p + 64 * k);
  }
  __device__ __forceinline__ f32x4 get(int k) const { return v[k]; }
};

// 16-bit stores: 4 features (8 B) per lane per k, widened exactly to f32 (Tensor.float()).
// Halves are taken one scalar at a time: a bit_cast of the two words to a _Float16 vector
// pair compiled (ROCm 7.2 clang) to code that converted the first word twice.
template <>
struct StoreRow<DAD_STORE_F16> {
  u32x2 v[3];
  __device__ __forceinline__ void load(const void* base, long frame, int lane) {
    const u32x2* p = reinterpret_cast<const u32x2*>(base) + (size_t)frame * (DAD_D / 4) + lane;
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = __builtin_nontemporal_load(p + 64 * k);
  }
  static __device__ __forceinline__ float h(uint32_t bits) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)bits);
  }
  __device__ __forceinline__ f32x4 get(int k) const {
    f32x4 r;
    r[0] = h(v[k][0] & 0xffffu); r[1] = h(v[k][0] >> 16); r[2] = h(v[k][1] & 0xffffu); r[3] = h(v[k][1] >> 16);
    return r;
  }
};

template <>
struct StoreRow<DAD_STORE_BF16> {
  u32x2 v[3];
  __device__ __forceinline__ void load(const void* base, long frame, int lane) {
    const u32x2* p = reinterpret_cast<const u32x2*>(base) + (size_t)frame * (DAD_D / 4) + lane;
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = __builtin_nontemporal_load(p + 64 * k);
  }
  __device__ __forceinline__ f32x4 get(int k) const {
    f32x4 r;   // bf16 -> f32 is the bf16 bits in the high half
    r[0] = __uint_as_float(v[k][0] << 16); r[1] = __uint_as_float(v[k][0] & 0xffff0000u);
    r[2] = __uint_as_float(v[k][1] << 16); r[3] = __uint_as_float(v[k][1] & 0xffff0000u);
    return r;
  }
};

template <int DT>
__device__ __forceinline__ void collate_body(const DadCollateArgs& a) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const long rows = (long)a.B * a.T;
  const long r0 = ((long)blockIdx.x * kWaves + wave) * kRowsPerWave;
  StoreRow<DT> sr[kRowsPerWave];
  bool live[kRowsPerWave];
#pragma unroll
  for (int i = 0; i < kRowsPerWave; ++i) {
    const long r = r0 + i;
    live[i] = false;
    if (r < rows) {
      const int b = (int)(r / a.T), t = (int)(r - (long)b * a.T);
      const long s = a.index[b];
      const bool ok = s >= 0 && s < a.n_samples;     // out of range -> an all-padding row
      const int size = ok ? a.sizes[s] : 0;
      live[i] = t < size;
      if (live[i]) sr[i].load(a.store, a.offsets[s] + t, lane);
      if (lane == 0) a.pad[r] = live[i] ? 0 : 1;     // I/dataload_noisy.py:127 padding_mask[i, size:] = True
    }
  }
#pragma unroll
  for (int i = 0; i < kRowsPerWave; ++i) {
    const long r = r0 + i;
    if (r >= rows) break;
    f32x4* dst = reinterpret_cast<f32x4*>(a.feats) + (size_t)r * (DAD_D / 4) + lane;
#pragma unroll
    for (int k = 0; k < 3; ++k) dst[64 * k] = live[i] ? sr[i].get(k) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // labels (I/dataload_clean.py:181 torch.tensor([s["target"] ...])) from the first workgroup
  if (blockIdx.x == 0 && a.labels_out)
    for (int b = threadIdx.x; b < a.B; b += DAD_COLLATE_THREADS) {
      const long s = a.index[b];
      a.labels_out[b] = (s >= 0 && s < a.n_samples) ? a.labels_in[s] : -1;
    }
}

}  // namespace

__global__ __launch_bounds__(DAD_COLLATE_THREADS) void dad_collate_kernel(DadCollateArgs a) {
  switch (a.dtype) {
    case DAD_STORE_F16: collate_body<DAD_STORE_F16>(a); break;
    case DAD_STORE_BF16: collate_body<DAD_STORE_BF16>(a); break;
    default: collate_body<DAD_STORE_F32>(a); break;
  }
}

// store-mode index: one thread per (b, t) pad byte; threads t == 0 also write row/len/label
__global__ __launch_bounds__(256) void dad_collate_index_kernel(DadCollateArgs a, int64_t* row_out, int32_t* len_out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)a.B * a.T) return;
  const int b = (int)(i / a.T), t = (int)(i - (long)b * a.T);
  const long s = a.index[b];
  const bool ok = s >= 0 && s < a.n_samples;
  const int size = ok ? a.sizes[s] : 0;
  a.pad[i] = t < size ? 0 : 1;
  if (t == 0) {
    row_out[b] = size > 0 ? a.offsets[s] : 0;     // an empty sample reads nothing past the store
    len_out[b] = size;
    if (a.labels_out) a.labels_out[b] = ok ? a.labels_in[s] : -1;
  }
}

// one block per sample of the epoch (samples in batch order): its pad row at pad_off[i], T = pad_T[i]
__global__ __launch_bounds__(256) void dad_collate_index_epoch_kernel(DadCollateArgs a, long n, const int64_t* pad_off,
                                                                     const int64_t* pad_T, int64_t* row_out,
                                                                     int32_t* len_out) {
  const long i = blockIdx.x;
  if (i >= n) return;
  const long s = a.index[i];
  const bool ok = s >= 0 && s < a.n_samples;
  const int size = ok ? a.sizes[s] : 0;
  const long T = pad_T[i];
  uint8_t* pad = a.pad + pad_off[i];
  for (long t = threadIdx.x; t < T; t += 256) pad[t] = t < size ? 0 : 1;
  if (threadIdx.x == 0) {
    row_out[i] = size > 0 ? a.offsets[s] : 0;
    len_out[i] = size;
    if (a.labels_out) a.labels_out[i] = ok ? a.labels_in[s] : -1;
  }
}

int dad_collate_grid(long B, long T) {
  const long per = (long)kWaves * kRowsPerWave;
  return (int)((B * T + per - 1) / per);
}

extern "C" int dad_collate(const void* store, int store_dtype, const int64_t* offsets, const int32_t* sizes,
                           int64_t n_samples, const int64_t* index, int B, int T, float* feats, uint8_t* pad,
                           const int64_t* labels_in, int64_t* labels_out, void* stream) {
  if (!store || !offsets || !sizes || !index || !feats || !pad) return DAD_E_ARG;
  if ((labels_in == nullptr) != (labels_out == nullptr)) return DAD_E_ARG;
  if (store_dtype != DAD_STORE_F32 && store_dtype != DAD_STORE_F16 && store_dtype != DAD_STORE_BF16) return DAD_E_ARG;
  if (B <= 0 || T <= 0 || n_samples <= 0) return DAD_E_SHAPE;
  DadCollateArgs a;
  a.store = store; a.dtype = store_dtype; a.offsets = offsets; a.sizes = sizes; a.n_samples = (long)n_samples;
  a.index = index; a.B = B; a.T = T; a.feats = feats; a.pad = pad;
  a.labels_in = labels_in; a.labels_out = labels_out;
  hipLaunchKernelGGL(dad_collate_kernel, dim3(dad_collate_grid(B, T)), dim3(DAD_COLLATE_THREADS), 0,
                     (hipStream_t)stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DAD_OK : (int)e;
}

extern "C" int dad_collate_index(const int64_t* offsets, const int32_t* sizes, int64_t n_samples, const int64_t* index,
                                 int B, int T, int64_t* row_out, int32_t* len_out, uint8_t* pad,
                                 const int64_t* labels_in, int64_t* labels_out, void* stream) {
  if (!offsets || !sizes || !index || !row_out || !len_out || !pad) return DAD_E_ARG;
  if ((labels_in == nullptr) != (labels_out == nullptr)) return DAD_E_ARG;
  if (B <= 0 || T <= 0 || n_samples <= 0) return DAD_E_SHAPE;
  DadCollateArgs a;
  memset(&a, 0, sizeof(a));
  a.offsets = offsets; a.sizes = sizes; a.n_samples = (long)n_samples; a.index = index; a.B = B; a.T = T;
  a.pad = pad; a.labels_in = labels_in; a.labels_out = labels_out;
  const long n = (long)B * T;
  hipLaunchKernelGGL(dad_collate_index_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a,
                     row_out, len_out);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DAD_OK : (int)e;
}

extern "C" int dad_collate_index_epoch(const int64_t* offsets, const int32_t* sizes, int64_t n_samples,
                                       const int64_t* index, int64_t n, const int64_t* pad_off, const int64_t* pad_T,
                                       int64_t* row_out, int32_t* len_out, uint8_t* pad, const int64_t* labels_in,
                                       int64_t* labels_out, void* stream) {
  if (!offsets || !sizes || !index || !pad_off || !pad_T || !row_out || !len_out || !pad) return DAD_E_ARG;
  if ((labels_in == nullptr) != (labels_out == nullptr)) return DAD_E_ARG;
  if (n <= 0 || n > (1L << 31) || n_samples <= 0) return DAD_E_SHAPE;
  DadCollateArgs a;
  memset(&a, 0, sizeof(a));
  a.offsets = offsets; a.sizes = sizes; a.n_samples = (long)n_samples; a.index = index;
  a.pad = pad; a.labels_in = labels_in; a.labels_out = labels_out;
  hipLaunchKernelGGL(dad_collate_index_epoch_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, a, (long)n,
                     pad_off, pad_T, row_out, len_out);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DAD_OK : (int)e;
}
