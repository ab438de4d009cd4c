// plan.h — host side of a handle's tone plan: which detector runs, the fp32
// constants its kernels read (the same arrays demod_create uploads), and the
// decision rescue's thresholds derived from those constants by a forward
// rounding-error analysis (error_model.cpp). No device calls:
// demod_error_model() evaluates it for a configuration without a GPU.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/demod.h"
#include "demod_internal.h"

namespace fskd {

struct Plan {
    int detector = kDetGoertzel;
    int log2g = 0;
    bool slide = false;          // n = 1024, hop = 64 H < n: segment-shared kernels (plain / fold)
    bool reinsch = false;        // plain bank: Reinsch-modified recurrence
    bool f16 = false;            // fold detector: fold by 16 (K = 8)
    int dcls = 0;                // residue detector: compile-time class pattern
    unsigned long long perm = 0; // DCLS / F16: nibble s = tone of kernel slot s
    int slot_tone[kMaxTones] = {};
    float coef[kMaxTones] = {};  // per kernel slot: 2 cos w (Reinsch: lambda)
    float sgn[kMaxTones] = {};
    int zcls[kMaxTones] = {};    // residue: class each slot reads
    std::vector<float4> rot;     // the rotation table as uploaded ([slot][g], residue [slot][g][2])
    double rcoef[kMaxTones] = {};  // 2 cos(2 pi f / fs) in double (the oracle's c), tone order
    int fft_bins[kMaxTones] = {};
    int fft_slot[kMaxTones] = {};
    std::vector<double> rot64;   // pass 0 tables (n = 1024, K >= 2): [k][16][4], then c[k]
    // pass 0 by the fold (1: every tone on a multiple of 8 bins): lane j's
    // chain runs over folded samples 8j .. 8j + 7 of the window folded to 128
    // (exact integer sums), rot64 = A = e^{-i w (8j + 7)}, B = e^{-i w (8j +
    // 8)} at the exact bin w = 2 pi b / n, c = 2 cos w; by the residue fold
    // (2: the residue detector's plans, every tone on an integer bin b): the
    // same positions of Y_rho = sum_m x[p + 128 m] e^{-2 pi i rho m / 8},
    // rho = b mod 8 (complex for odd / 2, 6 residues), its two real chains
    // and a complex rotation, rho after the coefficients in rot64; 0: lane
    // j's 64 raw samples (A = e^{-i w (64j + 63)}, ...)
    int fold64 = 0;
};

// DEMOD_OK or the error code demod_create returns for it.
int validate_cfg(const demod_cfg_t *c);
// Tone i's bin f_i n / fs if it is an integer (within rounding), else -1.
long long integer_bin(const demod_cfg_t &c, uint32_t i);
bool residue_eligible(const demod_cfg_t &c);  // every tone on an integer bin (residue.hip)
bool fold_eligible(const demod_cfg_t &c);     // ... on a multiple of 8 bins (fold.hip)

// Fills pl from a validated configuration.
void build_plan(const demod_cfg_t &c, Plan &pl);

// The rescue's thresholds. With E the energy the kernel's
// stage 2 sums (raw sum x^2; fold detector: sum xf^2 of the N/8-fold; FFT:
// Parseval's 2 sum_b P_b >= n sum x^2) a window is flagged when
//   (P_max - P_2nd)^2 < t2e E_eff P_max   (or P_max == 0 with E_eff > 0),
// E_eff = E, except the fold detector: (sqrt(E) + amb_d)^2 (the double
// oracle's own error scales with the raw window, which can hold energy the
// fold cancels). Stage 1 replaces E_eff by its int16 maximum: tq = sqrt(t2e
// E_max), fl = t2e E_max / 16.
struct ErrModel {
    double rho_det = 0;   // |sqrt(P_fp32) - |X|| <= rho_det sqrt(E_det), every tone
    double rho_ref = 0;   // |sigma(P_oracle) - |X|| <= rho_ref sqrt(sum x^2)
    double rho_first = 0; // pass 0: |sqrt(P_0) - sigma(P_oracle)| <= rho_first sqrt(sum x^2)
    double t2e = 0, tq = 0, fl = 0, amb_d = 0;
    double t2e64 = 0;     // pass 0's threshold, E its fp32 sum x^2 (0: off)
    double tau = 0;       // 4 (rho_det + rho_ref) / sqrt(n_eff): t2e = tau^2 n_eff
    double tau64 = 0;     // 4 rho_first / sqrt(n)
    int energy = 0;       // DEMOD_ENERGY_*
};

// fp32 detector + oracle bounds and the thresholds; first_pass: the handle
// runs pass 0 (n = 1024, K >= 2, not switched off).
void error_model(const demod_cfg_t &c, const Plan &pl, bool first_pass, ErrModel &m);

// demod_api.cpp helpers for demod_group.cpp: every argument refusal of
// demod_streams_push (its code) or the per-stream symbol counts the push
// emits (nullable counts; returns their total), and a streams handle's device
long long streams_check(const demod_streams_t *ms, const int16_t *const *pcm, const size_t *n_frames,
                        uint32_t *counts);
int streams_device(const demod_streams_t *ms);

}  // namespace fskd
