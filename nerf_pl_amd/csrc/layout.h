// Packed-weight and saved-activation layouts.  Mirrors nerf_pl_amd/packing.py
// (checked by tests/test_packing.py through nr_layout_query()).
#pragma once
#include "common.h"

// packed layer size in floats: ksteps * tiles * 64 lanes
#define NR_PL(ks, nt) ((ks) * (nt) * 64)

// ---- forward packed buffer -------------------------------------------------
#define NR_F_L1 0
#define NR_F_L2 (NR_F_L1 + NR_PL(32, 8))
#define NR_F_L3 (NR_F_L2 + NR_PL(128, 8))
#define NR_F_L4 (NR_F_L3 + NR_PL(128, 8))
#define NR_F_L5 (NR_F_L4 + NR_PL(128, 8))
#define NR_F_L6 (NR_F_L5 + NR_PL(160, 8))
#define NR_F_L7 (NR_F_L6 + NR_PL(128, 8))
#define NR_F_L8 (NR_F_L7 + NR_PL(128, 8))
#define NR_F_FINAL (NR_F_L8 + NR_PL(128, 8))
#define NR_F_DIR (NR_F_FINAL + NR_PL(128, 8))
#define NR_F_HEAD (NR_F_DIR + NR_PL(144, 4))
// head block (floats, relative to NR_F_HEAD)
#define NR_H_BIAS(l) (((l) - 1) * 256)   // l = 1..8
#define NR_H_BFINAL (8 * 256)
#define NR_H_BDIR (NR_H_BFINAL + 256)
#define NR_H_WSIG (NR_H_BDIR + 128)
#define NR_H_BSIG (NR_H_WSIG + 256)
#define NR_H_WRGB (NR_H_BSIG + 4)
#define NR_H_BRGB (NR_H_WRGB + 384)
#define NR_H_SIZE (NR_H_BRGB + 4)
#define NR_F_TOTAL (NR_F_HEAD + NR_H_SIZE)

// ---- backward (transposed) packed buffer ----------------------------------
#define NR_B_DIRT 0
#define NR_B_FINALT (NR_B_DIRT + NR_PL(64, 8))
#define NR_B_L8T (NR_B_FINALT + NR_PL(128, 8))
#define NR_B_L7T (NR_B_L8T + NR_PL(128, 8))
#define NR_B_L6T (NR_B_L7T + NR_PL(128, 8))
#define NR_B_L5T (NR_B_L6T + NR_PL(128, 8))
#define NR_B_L4T (NR_B_L5T + NR_PL(128, 8))
#define NR_B_L3T (NR_B_L4T + NR_PL(128, 8))
#define NR_B_L2T (NR_B_L3T + NR_PL(128, 8))
#define NR_B_TOTAL (NR_B_L2T + NR_PL(128, 8))

// ---- saved activations (forward, training mode) ---------------------------
// One buffer of NR_SAVE_PER_SAMPLE * n floats, segments row-major [n][width]:
//   pe[n][64] (paired k order: col 2g+h), h1..h8[n][256], feat[n][256],
//   hdir[n][128], dirpe[n][32] (paired k order)
#define NR_SAVE_PER_SAMPLE (64 + 8 * 256 + 256 + 128 + 32)
struct NrSave {
    float* pe; float* h[8]; float* feat; float* hdir; float* dirpe;
    __host__ __device__ NrSave(float* base, int64_t n) {
        pe = base;
        for (int l = 0; l < 8; ++l) h[l] = base + 64 * n + (int64_t)l * 256 * n;
        feat = base + 64 * n + 8 * 256 * n;
        hdir = feat + 256 * n;
        dirpe = hdir + 128 * n;
    }
};

// ---- per-layer pre-activation gradients (backward) ------------------------
//   dz1..dz8[n][256], dfeat[n][256], dzdir[n][128], dhead[n][4]=(drgb_z, dsigma)
#define NR_GRAD_PER_SAMPLE (8 * 256 + 256 + 128 + 4)
struct NrGrad {
    float* dz[8]; float* dfeat; float* dzdir; float* dhead;
    __host__ __device__ NrGrad(float* base, int64_t n) {
        for (int l = 0; l < 8; ++l) dz[l] = base + (int64_t)l * 256 * n;
        dfeat = base + 8 * 256 * n;
        dzdir = dfeat + 256 * n;
        dhead = dzdir + 128 * n;
    }
};
