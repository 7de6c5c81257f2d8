// ce_glibc_log.hpp -- glibc's f64 log, restated bit for bit for the device.
//
// Why: scipy.special.entr (amg_test.py:443, :451, :479 via scipy.stats.entropy)
// computes -x*log(x) with the C library's log, i.e. glibc's.  ocml's f64 log
// differs from it by up to 2 ulp on ~0.6 % of arguments, which could flip the
// order of two near-tied items at the q-th boundary.  With this routine every
// device entropy is the reference's entropy bit for bit.
//
// Algorithm: glibc >= 2.28 sysdeps/ieee754/dbl-64/e_log.c (ARM optimized-
// routines; glibc 2.35 in this image), as its x86-64 FMA ifunc variant
// (__log_fma, selected on every FMA-capable x86-64 host, the GPU box's EPYC
// included) evaluates it: the reduction is r = fma(z, invc, -1), and GCC's
// default contraction fuses every multiply whose only use is an add (the fma()
// calls below are exactly those).  Verified on the host against libm's log on
// 5e8 arguments (tests/test_glibc_log.py), and on the device against libm
// (tests/test_gpu_parity.py::test_device_log_bit_exact).
//   near 1 (1-2^-4 <= x < 1+0x1.09p-4): log1p polynomial of degree 11, with
//        the quadratic term split exactly (rhi has 26 significant bits);
//   else x = 2^k z, z in [0x1.6p-1, 0x1.6p0): 128-entry table {1/c, log c},
//        log x = k ln2 + log c + log1p(z/c - 1), degree-6 polynomial;
//   subnormals are scaled by 2^52 first; 0 -> -inf, inf -> inf, x<0 -> NaN.
// Table and coefficients: tools/gen_glibc_log_table.py (glibc's e_log_data.c
// constants as stored in libm).
//
// Device use: the 2 KB {invc, logc} table is staged into LDS once per block
// (stage_log_table(), before the first entropy) and read with one ds_read_b128
// per log -- a global table load would share vmcnt with the LDS-DMA / streaming
// loads in flight and serialise them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#define CE_GLIBC_LOG_LN2 0x1.62e42fefa3800p-1, 0x1.ef35793c76730p-45
#define CE_GLIBC_LOG_A -0x1.0000000000001p-1, 0x1.555555551305bp-2, -0x1.fffffffeb4590p-3, 0x1.999b324f10111p-3, -0x1.55575e506c89fp-3
#define CE_GLIBC_LOG_B -0x1.0000000000000p-1, 0x1.5555555555577p-2, -0x1.ffffffffffdcbp-3, 0x1.999999995dd0cp-3, -0x1.55555556745a7p-3, 0x1.24924a344de30p-3, -0x1.fffffa4423d65p-4, 0x1.c7184282ad6cap-4, -0x1.999eb43b068ffp-4, 0x1.78182f7afd085p-4, -0x1.5521375d145cdp-4
#define CE_GLIBC_LOG_TAB \
    0x1.734f0c3e0de9fp+0, -0x1.7cc7f79e69000p-2, 0x1.713786a2ce91fp+0, -0x1.76feec20d0000p-2, \
    0x1.6f26008fab5a0p+0, -0x1.713e31351e000p-2, 0x1.6d1a61f138c7dp+0, -0x1.6b85b38287800p-2, \
    0x1.6b1490bc5b4d1p+0, -0x1.65d5590807800p-2, 0x1.69147332f0cbap+0, -0x1.602d076180000p-2, \
    0x1.6719f18224223p+0, -0x1.5a8ca86909000p-2, 0x1.6524f99a51ed9p+0, -0x1.54f4356035000p-2, \
    0x1.63356aa8f24c4p+0, -0x1.4f637c36b4000p-2, 0x1.614b36b9ddc14p+0, -0x1.49da7fda85000p-2, \
    0x1.5f66452c65c4cp+0, -0x1.445923989a800p-2, 0x1.5d867b5912c4fp+0, -0x1.3edf439b0b800p-2, \
    0x1.5babccb5b90dep+0, -0x1.396ce448f7000p-2, 0x1.59d61f2d91a78p+0, -0x1.3401e17bda000p-2, \
    0x1.5805612465687p+0, -0x1.2e9e2ef468000p-2, 0x1.56397cee76bd3p+0, -0x1.2941b3830e000p-2, \
    0x1.54725e2a77f93p+0, -0x1.23ec58cda8800p-2, 0x1.52aff42064583p+0, -0x1.1e9e129279000p-2, \
    0x1.50f22dbb2bddfp+0, -0x1.1956d2b48f800p-2, 0x1.4f38f4734ded7p+0, -0x1.141679ab9f800p-2, \
    0x1.4d843cfde2840p+0, -0x1.0edd094ef9800p-2, 0x1.4bd3ec078a3c8p+0, -0x1.09aa518db1000p-2, \
    0x1.4a27fc3e0258ap+0, -0x1.047e65263b800p-2, 0x1.4880524d48434p+0, -0x1.feb224586f000p-3, \
    0x1.46dce1b192d0bp+0, -0x1.f474a7517b000p-3, 0x1.453d9d3391854p+0, -0x1.ea4443d103000p-3, \
    0x1.43a2744b4845ap+0, -0x1.e020d44e9b000p-3, 0x1.420b54115f8fbp+0, -0x1.d60a22977f000p-3, \
    0x1.40782da3ef4b1p+0, -0x1.cc00104959000p-3, 0x1.3ee8f5d57fe8fp+0, -0x1.c202956891000p-3, \
    0x1.3d5d9a00b4ce9p+0, -0x1.b81178d811000p-3, 0x1.3bd60c010c12bp+0, -0x1.ae2c9ccd3d000p-3, \
    0x1.3a5242b75dab8p+0, -0x1.a45402e129000p-3, 0x1.38d22cd9fd002p+0, -0x1.9a877681df000p-3, \
    0x1.3755bc5847a1cp+0, -0x1.90c6d69483000p-3, 0x1.35dce49ad36e2p+0, -0x1.87120a645c000p-3, \
    0x1.34679984dd440p+0, -0x1.7d68fb4143000p-3, 0x1.32f5cceffcb24p+0, -0x1.73cb83c627000p-3, \
    0x1.3187775a10d49p+0, -0x1.6a39a9b376000p-3, 0x1.301c8373e3990p+0, -0x1.60b3154b7a000p-3, \
    0x1.2eb4ebb95f841p+0, -0x1.5737d76243000p-3, 0x1.2d50a0219a9d1p+0, -0x1.4dc7b8fc23000p-3, \
    0x1.2bef9a8b7fd2ap+0, -0x1.4462c51d20000p-3, 0x1.2a91c7a0c1babp+0, -0x1.3b08abc830000p-3, \
    0x1.293726014b530p+0, -0x1.31b996b490000p-3, 0x1.27dfa5757a1f5p+0, -0x1.2875490a44000p-3, \
    0x1.268b39b1d3bbfp+0, -0x1.1f3b9f879a000p-3, 0x1.2539d838ff5bdp+0, -0x1.160c8252ca000p-3, \
    0x1.23eb7aac9083bp+0, -0x1.0ce7f57f72000p-3, 0x1.22a012ba940b6p+0, -0x1.03cdc49fea000p-3, \
    0x1.2157996cc4132p+0, -0x1.f57bdbc4b8000p-4, 0x1.201201dd2fc9bp+0, -0x1.e370896404000p-4, \
    0x1.1ecf4494d480bp+0, -0x1.d17983ef94000p-4, 0x1.1d8f5528f6569p+0, -0x1.bf9674ed8a000p-4, \
    0x1.1c52311577e7cp+0, -0x1.adc79202f6000p-4, 0x1.1b17c74cb26e9p+0, -0x1.9c0c3e7288000p-4, \
    0x1.19e010c2c1ab6p+0, -0x1.8a646b372c000p-4, 0x1.18ab07bb670bdp+0, -0x1.78d01b3ac0000p-4, \
    0x1.1778a25efbcb6p+0, -0x1.674f145380000p-4, 0x1.1648d354c31dap+0, -0x1.55e0e6d878000p-4, \
    0x1.151b990275fddp+0, -0x1.4485cdea1e000p-4, 0x1.13f0ea432d24cp+0, -0x1.333d94d6aa000p-4, \
    0x1.12c8b7210f9dap+0, -0x1.22079f8c56000p-4, 0x1.11a3028ecb531p+0, -0x1.10e4698622000p-4, \
    0x1.107fbda8434afp+0, -0x1.ffa6c6ad20000p-5, 0x1.0f5ee0f4e6bb3p+0, -0x1.dda8d4a774000p-5, \
    0x1.0e4065d2a9fcep+0, -0x1.bbcece4850000p-5, 0x1.0d244632ca521p+0, -0x1.9a1894012c000p-5, \
    0x1.0c0a77ce2981ap+0, -0x1.788583302c000p-5, 0x1.0af2f83c636d1p+0, -0x1.5715e67d68000p-5, \
    0x1.09ddb98a01339p+0, -0x1.35c8a49658000p-5, 0x1.08cabaf52e7dfp+0, -0x1.149e364154000p-5, \
    0x1.07b9f2f4e28fbp+0, -0x1.e72c082eb8000p-6, 0x1.06ab58c358f19p+0, -0x1.a55f152528000p-6, \
    0x1.059eea5ecf92cp+0, -0x1.63d62cf818000p-6, 0x1.04949cdd12c90p+0, -0x1.228fb8caa0000p-6, \
    0x1.038c6c6f0ada9p+0, -0x1.c317b20f90000p-7, 0x1.02865137932a9p+0, -0x1.419355daa0000p-7, \
    0x1.0182427ea7348p+0, -0x1.81203c2ec0000p-8, 0x1.008040614b195p+0, -0x1.0040979240000p-9, \
    0x1.fe01ff726fa1ap-1, 0x1.feff384900000p-9, 0x1.fa11cc261ea74p-1, 0x1.7dc41353d0000p-7, \
    0x1.f6310b081992ep-1, 0x1.3cea3c4c28000p-6, 0x1.f25f63ceeadcdp-1, 0x1.b9fc114890000p-6, \
    0x1.ee9c8039113e7p-1, 0x1.1b0d8ce110000p-5, 0x1.eae8078cbb1abp-1, 0x1.58a5bd001c000p-5, \
    0x1.e741aa29d0c9bp-1, 0x1.95c8340d88000p-5, 0x1.e3a91830a99b5p-1, 0x1.d276aef578000p-5, \
    0x1.e01e009609a56p-1, 0x1.07598e598c000p-4, 0x1.dca01e577bb98p-1, 0x1.253f5e30d2000p-4, \
    0x1.d92f20b7c9103p-1, 0x1.42edd8b380000p-4, 0x1.d5cac66fb5ccep-1, 0x1.606598757c000p-4, \
    0x1.d272caa5ede9dp-1, 0x1.7da76356a0000p-4, 0x1.cf26e3e6b2ccdp-1, 0x1.9ab434e1c6000p-4, \
    0x1.cbe6da2a77902p-1, 0x1.b78c7bb0d6000p-4, 0x1.c8b266d37086dp-1, 0x1.d431332e72000p-4, \
    0x1.c5894bd5d5804p-1, 0x1.f0a3171de6000p-4, 0x1.c26b533bb9f8cp-1, 0x1.067152b914000p-3, \
    0x1.bf583eeece73fp-1, 0x1.147858292b000p-3, 0x1.bc4fd75db96c1p-1, 0x1.2266ecdca3000p-3, \
    0x1.b951e0c864a28p-1, 0x1.303d7a6c55000p-3, 0x1.b65e2c5ef3e2cp-1, 0x1.3dfc33c331000p-3, \
    0x1.b374867c9888bp-1, 0x1.4ba366b7a8000p-3, 0x1.b094b211d304ap-1, 0x1.5933928d1f000p-3, \
    0x1.adbe885f2ef7ep-1, 0x1.66acd2418f000p-3, 0x1.aaf1d31603da2p-1, 0x1.740f8ec669000p-3, \
    0x1.a82e63fd358a7p-1, 0x1.815c0f51af000p-3, 0x1.a5740ef09738bp-1, 0x1.8e92954f68000p-3, \
    0x1.a2c2a90ab4b27p-1, 0x1.9bb3602f84000p-3, 0x1.a01a01393f2d1p-1, 0x1.a8bed1c2c0000p-3, \
    0x1.9d79f24db3c1bp-1, 0x1.b5b515c01d000p-3, 0x1.9ae2505c7b190p-1, 0x1.c2967ccbcc000p-3, \
    0x1.9852ef297ce2fp-1, 0x1.cf635d5486000p-3, 0x1.95cbaeea44b75p-1, 0x1.dc1bd3446c000p-3, \
    0x1.934c69de74838p-1, 0x1.e8c01b8cfe000p-3, 0x1.90d4f2f6752e6p-1, 0x1.f5509c0179000p-3, \
    0x1.8e6528effd79dp-1, 0x1.00e6c121fb800p-2, 0x1.8bfce9fcc007cp-1, 0x1.071b80e93d000p-2, \
    0x1.899c0dabec30ep-1, 0x1.0d46b9e867000p-2, 0x1.87427aa2317fbp-1, 0x1.13687334bd000p-2, \
    0x1.84f00acb39a08p-1, 0x1.1980d67234800p-2, 0x1.82a49e8653e55p-1, 0x1.1f8ffe0cc8000p-2, \
    0x1.8060195f40260p-1, 0x1.2595fd7636800p-2, 0x1.7e22563e0a329p-1, 0x1.2b9300914a800p-2, \
    0x1.7beb377dcb5adp-1, 0x1.3187210436000p-2, 0x1.79baa679725c2p-1, 0x1.377266dec1800p-2, \
    0x1.77907f2170657p-1, 0x1.3d54ffbaf3000p-2, 0x1.756cadbd6130cp-1, 0x1.432eee32fe000p-2

namespace ce {

struct LogEntry {
    double invc, logc;
};

// entries 0..127: glibc's {invc, logc}; entry 128: {A[1], A[3]}, the two
// polynomial coefficients the FMAs take as addends (kept next to the table so
// the device reads them with one LDS broadcast instead of rebuilding them in
// VGPRs for every log: gfx950's VOP3 reads at most one SGPR pair)
#define CE_GLIBC_LOG_DEFINE_TABLE(QUAL, NAME) \
    QUAL double NAME[258] = {CE_GLIBC_LOG_TAB, 0x1.555555551305bp-2, 0x1.999b324f10111p-3};
CE_GLIBC_LOG_DEFINE_TABLE(__device__ const, g_log_tab)
CE_GLIBC_LOG_DEFINE_TABLE(static const, h_log_tab)

__host__ __device__ __forceinline__ uint64_t dbits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
__host__ __device__ __forceinline__ double bitsd(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}

// glibc log(x); tab = the 128 {invc, logc} entries (LDS on the device).
__host__ __device__ __forceinline__ double glibc_log(double x, const LogEntry* tab) {
    constexpr double A[5] = {CE_GLIBC_LOG_A};
    constexpr double B[11] = {CE_GLIBC_LOG_B};
    constexpr double Ln2[2] = {CE_GLIBC_LOG_LN2};
    constexpr uint64_t LO = 0x3fee000000000000ull;  // asuint64(1.0 - 0x1p-4)
    constexpr uint64_t HI = 0x3ff1090000000000ull;  // asuint64(1.0 + 0x1.09p-4)
    constexpr uint64_t OFF = 0x3fe6000000000000ull;
    uint64_t ix = dbits(x);
    if (ix - LO < HI - LO) {
        if (ix == 0x3ff0000000000000ull) return 0.0;
        const double r = x - 1.0;
        const double r2 = r * r;
        const double r3 = r * r2;
        const double p =
            __builtin_fma(r3,
                          __builtin_fma(r3,
                                        __builtin_fma(r3, B[10], __builtin_fma(r2, B[9], __builtin_fma(r, B[8], B[7]))),
                                        __builtin_fma(r2, B[6], __builtin_fma(r, B[5], B[4]))),
                          __builtin_fma(r2, B[3], __builtin_fma(r, B[2], B[1])));
        double w = r * 0x1p27;
        const double rhi = r + w - w;
        const double rlo = r - rhi;
        w = rhi * rhi * B[0];  // exact: rhi has 26 bits, B[0] = -0.5
        const double hi = r + w;
        double lo = r - hi + w;
        lo = __builtin_fma(B[0] * rlo, rhi + r, lo);
        double y = __builtin_fma(r3, p, lo);  // y = r3*p; y += lo (contracted)
        return y + hi;
    }
    const uint32_t top = (uint32_t)(ix >> 48);
    if (top - 0x0010u >= 0x7ff0u - 0x0010u) {
        if ((ix << 1) == 0) return -__builtin_inf();
        if (ix == 0x7ff0000000000000ull) return x;
        if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return (x - x) / (x - x);
        ix = dbits(x * 0x1p52);  // subnormal: normalise
        ix -= 52ull << 52;
    }
    const uint64_t tmp = ix - OFF;
    const int i = (int)((tmp >> 45) % 128);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & (0xfffull << 52));
    const LogEntry e = tab[i];
    const double z = bitsd(iz);
    const double r = __builtin_fma(z, e.invc, -1.0);
    const double kd = (double)k;
    const double w = __builtin_fma(kd, Ln2[0], e.logc);
    const double hi = w + r;
    const double lo = __builtin_fma(kd, Ln2[1], w - hi + r);
    const double r2 = r * r;
    const double p = __builtin_fma(r2, __builtin_fma(r, A[4], A[3]), __builtin_fma(r, A[2], A[1]));
    const double y = __builtin_fma(r * r2, p, __builtin_fma(r2, A[0], lo));
    return y + hi;
}

// The same function, laid out for the device: the common case (x outside the
// near-1 window, positive, normal, finite -- every entropy term p of a row
// with more than one non-negligible class) is straight-line 32-bit integer +
// f64 FMA code; the near-1 window and the special inputs take glibc_log()
// above under a branch the whole wave usually skips.  Same bits as glibc_log
// for every input (the common-case operations are glibc_log's own).
// The common case only: x normal, positive and below the near-1 window
// (1 - 2^-4 = 0x3fee0000'00000000, whose low word is 0) -- every entropy term
// p < 0.9375.  Straight-line 32-bit integer + f64 FMA code, glibc_log's own
// operations for that case.
__host__ __device__ __forceinline__ bool glibc_log_common(double x) {
    return (uint32_t)(dbits(x) >> 32) - 0x00100000u < 0x3fee0000u - 0x00100000u;
}

__host__ __device__ __forceinline__ double glibc_log_core(double x, const LogEntry* tab) {
    constexpr double A[5] = {CE_GLIBC_LOG_A};
    constexpr double Ln2[2] = {CE_GLIBC_LOG_LN2};
    const uint64_t ix = dbits(x);
    const uint32_t hw = (uint32_t)(ix >> 32);
    const uint32_t thi = hw - 0x3fe60000u;                    // high word of ix - OFF (OFF's low word is 0)
    const int i = (int)((thi >> 13) & 127u);                  // (tmp >> 45) % 128
    const int k = (int)thi >> 20;                             // (int64_t)tmp >> 52
    const uint32_t izh = hw - (thi & 0xfff00000u);            // ix - (tmp & 0xfff << 52)
    const double z = bitsd(((uint64_t)izh << 32) | (uint32_t)ix);
    const LogEntry e = tab[i];
    const double r = __builtin_fma(z, e.invc, -1.0);
    const double kd = (double)k;
    const double w = __builtin_fma(kd, Ln2[0], e.logc);
    const double hi = w + r;
    const double lo = __builtin_fma(kd, Ln2[1], w - hi + r);
    const double r2 = r * r;
    const LogEntry a13 = tab[128];  // {A[1], A[3]}
    const double p = __builtin_fma(r2, __builtin_fma(r, A[4], a13.logc), __builtin_fma(r, A[2], a13.invc));
    return __builtin_fma(r * r2, p, __builtin_fma(r2, A[0], lo)) + hi;
}

// The same function as glibc_log for every input, laid out for the device:
// the common case straight-line, everything else (near 1, above it,
// subnormal, zero, negative, inf, NaN) through glibc_log under a branch the
// wave usually skips.
__host__ __device__ __forceinline__ double glibc_log_fast(double x, const LogEntry* tab) {
    if (__builtin_expect(!glibc_log_common(x), 0)) return glibc_log(x, tab);
    return glibc_log_core(x, tab);
}

// The block's LDS copy of the table (every kernel that computes an entropy
// calls stage_log_table() at its top, before any early exit).
__shared__ __attribute__((aligned(16))) LogEntry s_log_tab[129];

__device__ __forceinline__ const LogEntry* stage_log_table() {
    for (int j = threadIdx.x; j < 129; j += blockDim.x)
        s_log_tab[j] = LogEntry{g_log_tab[2 * j], g_log_tab[2 * j + 1]};
    __syncthreads();
    return s_log_tab;
}
__device__ __forceinline__ double dlog(double x) { return glibc_log_fast(x, s_log_tab); }

// Split staging for latency-bound kernels: fetch() issues the table loads at
// kernel start (before the data loads), commit() -- once the data has been
// waited for anyway -- writes them to LDS and syncs the block (block-uniform).
// Needs blockDim.x >= 129.
struct LogTablePrefetch {
    double invc, logc;
    __device__ __forceinline__ void fetch() {
        const int j = threadIdx.x < 129 ? threadIdx.x : 128;
        invc = g_log_tab[2 * j];
        logc = g_log_tab[2 * j + 1];
    }
    __device__ __forceinline__ void commit() const {
        if (threadIdx.x < 129) s_log_tab[threadIdx.x] = LogEntry{invc, logc};
        __syncthreads();
    }
};

inline const LogEntry* host_log_table() { return reinterpret_cast<const LogEntry*>(h_log_tab); }

}  // namespace ce
