// common.hpp — shared host/device helpers for the MI355X ANN search backend.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>
#include <cstdio>

namespace hipann {

// The IVF plan's per-query count step, handed to the coarse quantizer's probe select (runtime.hpp
// FlatShard::plan_hook, rows_select_small): list counts into ccnt, per-query slot prefixes and totals.
// The IVF query-major plan's per-list counts and fill cursors are kept in kPlanCopies copies ([copy][list]), query q
// counting into copy q % kPlanCopies: the coarse select's count step and the fill issue one atomic per (query,
// probe), and a popular list's atomics all landing on one word serialise at the memory side (≈7 µs of the
// 1024-query count step at 10M x 768).  The plan sums the copies; copy c's rows of a list's bucket start after
// copies 0..c-1.
constexpr int kPlanCopies = 8;
struct IvfPlanHook {
    const int *list_len;
    int nlist, chunk_rows;
    int *ccnt, *slot_off, *qtot;
    bool done;
};

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define HIPANN_CHECK(expr)                                                                             \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess) {                                                                        \
            throw ::hipann::HipError(std::string(#expr) + " failed: " + hipGetErrorString(_e) + " (" + \
                                     __FILE__ + ":" + std::to_string(__LINE__) + ")");                 \
        }                                                                                              \
    } while (0)

#define HIPANN_REQUIRE(cond, msg)                                        \
    do {                                                                 \
        if (!(cond)) throw ::hipann::HipError(std::string("hipann: ") + (msg)); \
    } while (0)

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Metric codes of the C ABI (hip_ann.h / hip_diskann_bridge.h).
enum Metric : int { kL2 = 0, kIP = 1 };
// IVF list-scan distance form (hipann_ivf_set_form): ‖q‖²+‖x‖²−2q·x (FAISS GPU / faiss-metal IVF) on the
// matrix cores, or the direct Σ(q−x)² of FAISS's CPU IndexIVFFlat scanner.
// kFormDecomposedValu: the same form on the VALU kernel (ivf_scan_dot), kept for A/B measurement.
// kFormSplit3 / kFormSplit2: the decomposed form on the bf16 matrix cores over a 3-term (fp32-level
// products) / 2-term bf16 split of both operands (ivf_mfma.hip, split-bf16 variant).
// kFormSplit2Exact: the 2-term scan keeps the kRerankK best per list and every returned distance is
// recomputed exactly in the direct form, with a per-query bound check (ivf_rerank_topk); k <= kRerankMaxK.
// kFormHalfExact (default): the same filter + rerank, the scan over a tiled fp16 image of the rows (half
// the bytes of the fp32 forms) with 2-term fp16 queries; the bound uses the measured fp16 residuals.
enum IvfForm : int {
    kFormDecomposed = 0,
    kFormDirect = 1,
    kFormDecomposedValu = 2,
    kFormSplit3 = 3,
    kFormSplit2 = 4,
    kFormSplit2Exact = 5,
    kFormHalfExact = 6,
    // kFormI8Exact (opt-in): the same filter + rerank over a tiled int8 image with one scale per row (a quarter of the
    // fp32 rows' bytes), sub-lists always, the rerank certified with the int8 residuals
    kFormI8Exact = 7
};
constexpr int kRerankK = 16, kRerankMaxK = 12;
// request_k in (kRerankMaxK, kIvfSubMaxK] on the IVF exact forms: sub-list slots (one 16-list per scan wave) and a
// rerank filter of min(64, max(kout + 4, 2·kout)) candidates (ivf.cpp); above: the 3-term scan
constexpr int kIvfSubMaxK = 60;
// Flat exact form, IP: 32 candidates per (split, query).  At 10M × 768 (U(-1,1) rows) 16 left ≈0.2% of
// the IP queries failing the bound (each a re-scan of the shard: 61 → 67 ms per batch), 32 none (65 ms);
// L2 had no failures at 16, and 32 costs it 60 → 66 ms (the fuller epilogue lists), so L2 keeps 16.
constexpr int kFlatRerankKIP = 32;
// Flat BLAS-path (nq >= kBlasThreshold) q·x form (hipann_flat_set_form): exact fp32 MFMA products
// (flat_gemm_topk2), or the fp32-level 3-term split-bf16 products on the bf16 matrix cores
// (flat_gemm_topk_bf); kFlatSplit2 is the 2-term split (≈2^-16 relative, A/B only).  kFlatSplit2Exact
// (default): the 2-term scan keeps kRerankK rows per database split and query as a filter, every
// returned distance is recomputed exactly in the direct form with the IVF exact form's bound check
// (ivf_rerank_topk), failures re-run on kFlatSplit3; kout <= kRerankMaxK (else kFlatSplit3).
// kFlatBf16Exact: the same filter + rerank on ONE plain bf16 product per element (flat_bf16.hip:
// a tiled bf16 image of the database built once; 32 kept per (split, query); the rerank's bound is the
// Cauchy-Schwarz bound of the actual bf16 rounding residuals), failures re-run on kFlatSplit3.
// kFlatI8Exact (default; shapes the bounded passes do not take fall back to kFlatBf16Exact): the same bounded
// passes over a tiled int8 image (per-row scale max|x|/127) on the int8 matrix
// cores (int32 sums: exact; twice the bf16 rate and half its bytes); the bound uses the int8 residuals.
enum FlatForm : int {
    kFlatFp32 = 0,
    kFlatSplit3 = 1,
    kFlatSplit2 = 2,
    kFlatSplit2Exact = 3,
    kFlatBf16Exact = 4,
    kFlatI8Exact = 5
};
// rerank bound E = eps·(‖q‖² + max‖x‖²) of the 2-term split scans' filters
constexpr float kSplit2Eps = 0x1p-12f;
__host__ __device__ inline bool ivf_form_split(int f) { return f == kFormSplit3 || f == kFormSplit2; }
__host__ __device__ inline int ivf_form_terms(int f) { return f == kFormSplit3 ? 3 : 2; }

// Query groups of an IVF list probed by c queries.  `group` packs the scan's group sizes: narrow (bits 0-7), wide
// (bits 8-15, 0 = none) and GEMM (bits 16-27, 0 = none).  A list probed by more queries than the narrow size is
// scanned in groups of up to the wide size (the fp16 scan's one-term items, ivf_mfma.hip), and one probed by more
// than the wide size in groups of up to the GEMM size (the GEMM-shaped items), so its rows are streamed ceil(c / size)
// times.  A narrow size of 0 makes every probed list at least wide (the default of the fp16 form).
__host__ __device__ inline int ivf_group_narrow(int group) { return group & 0xff; }
__host__ __device__ inline int ivf_group_wide(int group) { return (group >> 8) & 0xff; }
__host__ __device__ inline int ivf_group_gemm(int group) { return group >> 16; }
// 0 narrow, 1 wide, 2 GEMM
__host__ __device__ inline int ivf_list_class(int c, int group) {
    const int n = ivf_group_narrow(group), w = ivf_group_wide(group), m = ivf_group_gemm(group);
    if (m > 0 && c > (w > 0 ? w : n)) return 2;
    return w > 0 && c > n ? 1 : 0;
}
__host__ __device__ inline bool ivf_list_wide(int c, int group) { return ivf_list_class(c, group) == 1; }
__host__ __device__ inline int ivf_ngroups(int c, int group) {
    if (c <= 0) return 0;  // (an unprobed list: no division by a zero narrow size)
    const int cls = ivf_list_class(c, group);
    const int g = cls == 2 ? ivf_group_gemm(group) : cls == 1 ? ivf_group_wide(group) : ivf_group_narrow(group);
    return (c + g - 1) / g;
}
// the smallest group size (the work-item bound)
__host__ __device__ inline int ivf_group_min(int group) {
    return ivf_group_narrow(group) > 0 ? ivf_group_narrow(group) : ivf_group_wide(group);
}

// XCD-aware block remap (cdna_hip_programming.md §5.5 T1, bijective form): blocks b and b+8 are
// dealt to the same XCD; map so that each XCD receives a contiguous run of logical blocks.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
    const int q = nblocks >> 3, r = nblocks & 7;
    const int xcd = bid & 7, j = bid >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
}

}  // namespace hipann
