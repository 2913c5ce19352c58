// ldpc_bs.hip — host side of the bit-sliced fused QMS decoder (kernel: ldpc_bs_kernel.h, one
// instance per translation unit: ldpc_bs_inst.hip): instance choice, LDS layout, graph tables,
// per-decode weight tables, launch.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "ldpc_bs_kernel.h"

namespace ldpc {
namespace bs {

// per-decode tables: 16-entry g(m) tables as mux-tree leaves, [t][table][bit j][pair p] {X, Y}
// with Y = bit j of g(2p) (as a 0 / ~0 word) and X = Y ^ (bit j of g(2p + 1)):
// level 1 of the tree is (m0 & X) ^ Y.
//   alpha: g(m) = Q(relu(fl32(min(m, qmax) step * alpha_{t,row}))) (Main_Functions.py:266-316),
//          m = min(|V->C|) saturated at 15 (see bs_qmax);
//          with UCN the alpha' tables (rows arows .. 2 arows - 1) follow the alpha ones
//   beta:  g(m) = Q(fl32(m * beta_{t,col})) in grid units (lw = Q(beta ch), :164-177; beta >= 0),
//          then 4 words: the planes of |Q(fl32(cu * beta))| for a shortened bit (|ch| = cu)
__global__ void k_bs_tables(const float* __restrict__ alpha, const float* __restrict__ alpha_ucn,
                            const float* __restrict__ beta, const int32_t* __restrict__ row_ptr,
                            int T, int E, int N, int arows, int ar, int bcols, float step, float inv,
                            int qmax, float cu, uint32_t* alut, uint32_t* blut, int32_t* atid) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;    // one table per thread
    const int na = T * ar, nbt = T * bcols;
    if (f >= na + nbt) return;
    int g[16];
    uint32_t* out;
    if (f < na) {
        const int t = f / ar, r = f - t * ar;
        const float* al = (r < arows) ? alpha : alpha_ucn;
        const int row = (r < arows) ? r : r - arows;
        const float w = al[(size_t)t * E + row_ptr[row]];
        for (int m = 0; m < 16; ++m) g[m] = f5::q_mag5(min(m, qmax), w, step, inv, qmax);
        out = alut + (size_t)f * LUT_W;
        // the table's index in the fixed set (ldpc_beta_tabs.h), -1 if it is not one of them:
        // the kernels evaluate a table of the set with immediate truth tables (table_asm2)
        int id = -1;
        if (qmax == QMAX) {
            int sum = 0;
            for (int m = 0; m < 16; ++m) sum += g[m];
            for (int k = 0; k < kNBetaTab && id < 0; ++k) {
                bool eq = true;
                int sk = 0;
                for (int m = 0; m < 16; ++m) sk += kBetaTab[k][m];
                if (sk != sum) continue;
                for (int m = 0; m < 16; ++m) eq = eq && kBetaTab[k][m] == g[m];
                if (eq) id = k;
            }
        }
        atid[f] = id;
    } else {
        const int f2 = f - na;
        const int t = f2 / bcols, col = f2 - t * bcols;
        const float b = beta[(size_t)t * N + col];
        for (int m = 0; m < 16; ++m) {
            const int q = (int)__builtin_amdgcn_fmed3f(rintf((float)m * b), -(float)qmax, (float)qmax);
            g[m] = q < 0 ? -q : q;       // beta >= 0 (checked on the host)
        }
        out = blut + (size_t)f2 * BLUT_W;
        const int qb = (int)__builtin_amdgcn_fmed3f(rintf(cu * b), -(float)qmax, (float)qmax);
        for (int j = 0; j < 4; ++j) out[LUT_W + j] = (((qb < 0 ? -qb : qb) >> j) & 1) ? ~0u : 0u;
    }
    for (int j = 0; j < 4; ++j)
        for (int p = 0; p < 8; ++p) {
            const uint32_t y = ((g[2 * p] >> j) & 1) ? ~0u : 0u;
            const uint32_t x = y ^ (((g[2 * p + 1] >> j) & 1) ? ~0u : 0u);
            out[j * 16 + 2 * p] = x;
            out[j * 16 + 2 * p + 1] = y;
        }
}

// ---- host: planning, graph tables, launch -------------------------------------------------
typedef int (*LaunchFn)(const BsArgs&, int, int, size_t, hipStream_t, bool);
template <int... I>
constexpr auto launch_table(std::integer_sequence<int, I...>) {
    return std::array<LaunchFn, sizeof...(I)>{&bs_launch<I>...};
}

struct BsPlan {
    bool ok = false;
    int inst = -1, nw = 0, cn_lanes = 0, arows = 1, bcols = 1;
    uint32_t off_slots = 0, off_pad = 0, off_zero = 0, off_red = 0, off_alut = 0, off_blut = 0, off_hdz = 0,
             off_btid = 0, off_ch = 0, off_hdl = 0, off_preb = 0;
    int cn_dmin = 0;
    bool ucn = false;
    bool colalign = false;         // variable lanes: each column on a half-wave of its own
    float cu = 0.f;
    size_t lds = 0;
    std::vector<int32_t> lay;      // [M][2] first slot of proto row i, stride A_i of its j-blocks
};

// Column-aligned variable lanes (the one-chunk instances, z <= 32): the variables of each column
// start a 32-lane half-wave of their own (32 - z idle lanes after them).  Edge f of the z
// variables of one column reads the slots first + (k mod LPC) A + (k div LPC) z + (hh - shift)
// mod z: z consecutive slots, distinct mod 32, so every half-wave slot read of the variable phase
// is free of bank conflicts; packed, a half-wave holds the tail of one column and the head of
// the next, whose runs overlap mod 32 (802.11n, z = 27: 143 bank cycles per slot word in the
// bank model against a floor of 78, tools/bank_model.py).  Taken when it costs at most one more
// wave than the packed lanes (802.11n: 12 waves against 11; wman, z = 24, would need 12 against
// 9).  LDPC_BS_COLALIGN=0/1 forces it off / on where it fits.
static bool colalign_fits(const host::GraphTables& h, int nw_packed) {
    return h.z <= 32 && 32 * h.N <= 64 * 16 && (32 * h.N + 63) / 64 <= nw_packed + 1;
}

// Slot layout: edge k of check (row i, index h) is slot first_i + (k mod LPC) A_i +
// (k div LPC) z + h.  LDS banking (MI355X_MICROARCH.md, LDS): ds_read_b32 / ds_read2_b32 /
// ds_write_b32 serve a wave in two 32-lane groups, bank = dword address mod 32; a slot's words
// are 5 s + p (the slot array starts at a multiple of 128 B), so a group is conflict-free when
// its 32 slot numbers are distinct mod 32.  The 32 / LPC consecutive checks of a group read, for
// one m, slots first + j A + h: with first_i = first_{i-1} + z (mod 32) the checks stay
// consecutive mod 32 across a row boundary, and A_i is the smallest stride >= the j = 0 block
// whose multiples j A_i (j < LPC) are at least 32 / LPC apart mod 32.
std::vector<int32_t> slot_layout_rows(const host::GraphTables& h, const std::vector<int>& rl, size_t* nslot) {
    std::vector<int32_t> lay((size_t)2 * h.M, 0);
    size_t cur = 0;
    for (int i = 0; i < h.M; ++i) {
        const int LPC = rl[(size_t)i], sep = 32 / LPC;
        auto ok = [&](int A) {
            for (int d = 1; d < LPC; ++d) {
                const int r = (d * A) % 32;
                if (std::min(r, 32 - r) < sep) return false;
            }
            return true;
        };
        const int deg = h.row_ptr[i + 1] - h.row_ptr[i];
        size_t first = cur;
        if (i > 0) first += (size_t)((((int64_t)lay[2 * (i - 1)] + h.z - (int64_t)cur) % 32 + 32) % 32);
        int A = ((deg + LPC - 1) / LPC) * h.z;
        while (!ok(A)) ++A;
        const int last_rows = (deg - (LPC - 1) + LPC - 1) / LPC;   // block j = LPC - 1
        cur = first + (size_t)(LPC - 1) * A + (size_t)std::max(last_rows, 0) * h.z;
        lay[2 * i] = (int32_t)first;
        lay[2 * i + 1] = A;
    }
    *nslot = cur;
    return lay;
}
std::vector<int32_t> slot_layout(const host::GraphTables& h, int LPC, size_t* nslot) {
    return slot_layout_rows(h, std::vector<int>((size_t)h.M, LPC), nslot);
}

// The QMS grids both bit-sliced kernels decode: q = 5 (step 0.5), -5 (1), 4 (1), 3 (2), values
// |m| <= qmax in grid units (Cal_MSA_Q, Print_Functions.py:12-25; Main_Functions.py:475-494).
// Messages keep four magnitude planes saturated at 15 >= qmax: a V->C magnitude only reaches the
// check's two minima and the [|V->C| = min] test, and the alpha tables are built on
// min(m, qmax), so saturating at 15 instead of qmax leaves every C->V unchanged (the clamp
// commutes with the order statistics, and whenever the minimum is >= qmax every edge gets
// g(qmax)); APP and Tv are sums of C->V and the channel, which is checked against qmax.
bool bs_mode(int mode) { return mode == MODE_Q5 || mode == MODE_QM5 || mode == MODE_Q4 || mode == MODE_Q3; }
float bs_step(int mode) { return mode == MODE_Q5 ? 0.5f : mode == MODE_Q3 ? 2.0f : 1.0f; }
int bs_qmax(int mode) { return mode == MODE_Q4 ? 7 : mode == MODE_Q3 ? 3 : QMAX; }
static float mode_step_bs(int mode) { return bs_step(mode); }

// the plan of one instance (ok = it serves the graph)
static BsPlan plan_inst(const DevGraph& g, int i, bool ucn, float clip, int min_cdeg, int mode, int T) {
    BsPlan p;
    const BsInst& k = kBsInst[i];
    const host::GraphTables& h = *g.host;
    if (h.max_cdeg > k.D || h.max_vdeg > k.DV || (ucn && !k.UCN)) return p;
    p.inst = i;
    p.ucn = ucn;
    const int nv = g.n_vars, nc = g.n_checks;
    p.cn_lanes = 64 * ((k.LPC * nc + 63) / 64);
    int vch = (nv + 63) / 64;
    const int cch = p.cn_lanes / 64;
    if (k.VPL == 1 && k.CPL == 1) {
        static const int eca = [] { const char* e = getenv("LDPC_BS_COLALIGN"); return e ? atoi(e) : BS_COLALIGN; }();
        p.colalign = eca != 0 && colalign_fits(h, std::max(vch, cch));
        if (p.colalign) vch = (32 * h.N + 63) / 64;
    }
    if (k.VPL == 1 && k.CPL == 1) p.nw = std::max(vch, cch);
    else p.nw = std::max((vch + k.VPL - 1) / k.VPL, (cch + k.CPL - 1) / k.CPL);
    if (p.nw > 16) return p;                       // 1024-lane workgroup
    if (k.VPL > 1 || k.CPL > 1) {
        // spread over NW waves (one workgroup per CU); the chunks are dealt to the SIMDs
        p.nw = k.NW;
        if (vch > k.VPL * p.nw || cch > k.CPL * p.nw) return p;
    }
    // (one alpha / alpha' per iteration: one table pair, read by every lane at the same address,
    // a broadcast; per-row copies of it put the rows' tables in the same banks)
    const char* eap = getenv("LDPC_BS_AROWS");
    p.arows = ((g.w_alpha_uniform && !ucn) || (g.w_alpha_pair_uniform && !(eap && atoi(eap) == 0))) ? 1 : h.M;
    p.bcols = g.w_beta_uniform ? 1 : h.N;
    // idle check lanes: every slot is decided per lane
    p.cn_dmin = (p.cn_lanes == k.LPC * nc) ? min_cdeg : 0;
    if (k.BIG) {
        const float cu = clip / mode_step_bs(mode);
        if (cu > (float)bs_qmax(mode)) p.cu = cu;
    }
    size_t nslot = 0;
    p.lay = slot_layout(h, k.LPC, &nslot);
    // LDS: [UCN: hard decisions HD[nv], the zero word] | slots | PAD | ZERO | RED | ALUT | BLUT
    size_t o = 0;
    if (k.UCN) {
        p.off_hdz = (uint32_t)(4 * (size_t)nv);
        o = ((size_t)4 * (nv + 1) + 127) & ~(size_t)127;
    }
    p.off_slots = (uint32_t)o;
    p.off_pad = (uint32_t)(o + nslot * SLOT_B);
    p.off_zero = p.off_pad + SLOT_B;
    const size_t slot_end = (size_t)p.off_zero + SLOT_B;
    if (k.PK && slot_end > 65535) return p;        // 16-bit slot addresses
    if (k.UCN && p.off_hdz > 65535) return p;
    o = (slot_end + 15) & ~(size_t)15;
    p.off_red = (uint32_t)o;
    // + the per-iteration frame-error words, rounded to 16 B: the tables after them are read
    // with ds_read_b128 (T = 50 unrounded put them 8 B off: C3 17.8 -> 24.4 ms, C5 61 -> 81 ms)
    // and the 32 words the variable phases OR their frame-error words into (BS_FLOR)
    o += 64 + (((size_t)4 * T + 15) & ~(size_t)15) + 4 * BS_FLORW;
    p.off_alut = (uint32_t)o;
    o += (size_t)2 * (k.UCN ? 2 : 1) * p.arows * LUT_W * 4;
    p.off_blut = (uint32_t)o;
    o += (size_t)2 * p.bcols * BLUT_W * 4;
    if (k.PK && k.CPL == 1 && o > 65535) return p;  // 16-bit alpha-table addresses (BS_PKG)
    p.off_btid = (uint32_t)o;                      // the next iteration's channel-table ids
    o += ((size_t)4 * p.bcols + 15) & ~(size_t)15;
    if (BS_CH_LDS) {                               // the channel planes, 16 B per (lane, variable)
        p.off_ch = (uint32_t)o;
        o += (size_t)16 * k.VPL * 64 * p.nw;
    } else if (BS_GBLDS && k.CPL == 1) {           // the check lanes' slot-base words
        p.off_ch = (uint32_t)o;                    // (BS_ALDS: + their slot addresses, 2 per word)
        const int EPL = (k.D + k.LPC - 1) / k.LPC;
        o += (size_t)4 * (BS_ALDS && k.PK ? ((1 + (EPL + 1) / 2) | 1) : 1) * 64 * p.nw;
    }
    if (BS_HDLDS && k.UCN && k.CPL == 1) {         // the check lanes' hard-decision addresses
        const int EPL = (k.D + k.LPC - 1) / k.LPC, HDW = (EPL + 1) / 2;
        p.off_hdl = (uint32_t)o;
        o += (size_t)4 * HDW * 64 * p.nw;
    }
    // the check-idle waves' next channel tables (PREB, ldpc_bs_kernel.h): 16 B per lane of the
    // waves past cn_lanes
    const bool preb = (BS_PREB < 0 ? (k.UCN && k.VPL == 1 && k.CPL == 1) : BS_PREB != 0) && k.VPL == 1 &&
                      k.CPL == 1 && !BS_BTID_LDS;
    if (preb && p.nw * 64 > p.cn_lanes) {
        o = (o + 15) & ~(size_t)15;
        p.off_preb = (uint32_t)o;
        o += (size_t)16 * (64 * p.nw - p.cn_lanes);
    }
    p.lds = (o + 15) & ~(size_t)15;
    if (p.lds > BS_LDS_MAX) return p;
    p.ok = true;
    return p;
}

BsPlan bs_plan(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T) {
    BsPlan p;
    const char* e = getenv("LDPC_BS");
    if (e && atoi(e) == 0) return p;
    const char* el = getenv("LDPC_BS_LPC");          // A/B: force 2 or 4 lanes per check
    const int want_lpc = el ? atoi(el) : 0;
    const char* ei = getenv("LDPC_BS_INST");         // A/B: force one instance (if it fits)
    const int want_inst = ei ? atoi(ei) : -1;
    if (!bs_mode(mode)) return p;
    if (per_edge_w || !g.host || !g.w_beta_nonneg) return p;
    const host::GraphTables& h = *g.host;
    int min_cdeg = 1 << 30;
    for (int i = 0; i < h.M; ++i) min_cdeg = std::min(min_cdeg, h.row_ptr[i + 1] - h.row_ptr[i]);
    if (min_cdeg < 2) return p;                                   // ("no other edge" rule unneeded)
    for (int i = 0; i < kBsNInst; ++i) {
        if (want_lpc != 0 && want_lpc != kBsInst[i].LPC) continue;
        if (want_inst >= 0 && want_inst != i) continue;
        if (want_inst < 0 && kBsInst[i].NW != 16 && (kBsInst[i].VPL > 1 || kBsInst[i].CPL > 1)) continue;   // A/B only
        BsPlan q = plan_inst(g, i, ucn, clip, min_cdeg, mode, T);
        if (q.ok) return q;
    }
    return p;
}

}  // namespace bs

using namespace bs;

bool bs_supported(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T) {
    return bs_plan(g, mode, ucn, per_edge_w, clip, T).ok || bsc_supported(g, mode, ucn, per_edge_w, clip, T);
}

const char* bs_kernel_name(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T) {
    static thread_local char buf[64];
    const BsPlan p = bs_plan(g, mode, ucn, per_edge_w, clip, T);
    if (!p.ok) return bsc_kernel_name(g, mode, ucn, per_edge_w, clip, T);
    const BsInst& k = kBsInst[p.inst];
    if (k.VPL == 1 && k.CPL == 1)
        snprintf(buf, sizeof(buf), "bsl[p32,w%d,d%d,v%d,l%d%s]", p.nw, k.D, k.DV, k.LPC, p.ucn ? ",ucn" : "");
    else
        snprintf(buf, sizeof(buf), "bsl[p32,w%d,d%d,v%d,l%d,x%d/%d%s]", p.nw, k.D, k.DV, k.LPC, k.VPL,
                 k.CPL, p.ucn ? ",ucn" : "");
    return buf;
}

namespace bs {
// Deal `n` chunks (costs `cost`) to nw waves with at most `cap` chunks per wave (slot[w][c] =
// chunk or -1; wave w runs on SIMD w mod 4).  The chunks of one phase end at a barrier, and a
// SIMD's last busy wave runs alone, latency-bound (a dependent chain issues every ~8.5 cycles
// against ~2.4-4.2 with several waves), so what bounds a phase is the SIMD's total AND its
// heaviest wave.  Chunks go heaviest first to the lightest wave with room (LPT: 5G BG2's 20
// variable chunks on 16 waves pair the four lightest, 4 + 4 units, where the SIMD-first dealing
// gave one wave per SIMD 11 + 4 while the others held 4-7); the waves then go heaviest first
// to the SIMD with the smallest total and a free wave slot.  A wave's chunks are in descending
// cost (the first place takes the heaviest: bsc's heavy-degree place).  LDPC_BS_DEAL=0: the
// previous dealing (heaviest chunk to the least-loaded SIMD, on its emptiest wave).
// the exact dealing for the one-chunk instances (same box, r6c: C2 4.482 -> 4.458 ms over three
// rounds; C3's chunks are all but two of one cost, its deal unchanged)
#ifndef BS_DEAL_DEFAULT
#define BS_DEAL_DEFAULT 2
#endif
std::vector<int> deal_chunks(const std::vector<int>& cost, int nw, int cap) {
    const int n = (int)cost.size();
    std::vector<int> order(n), slot((size_t)nw * cap, -1);
    for (int c = 0; c < n; ++c) order[c] = c;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return cost[x] > cost[y]; });
    const char* e = getenv("LDPC_BS_DEAL");
    if (e && atoi(e) == 0) {
        std::vector<int> used(nw, 0), load(4, 0);
        for (int c : order) {
            int best = -1, bw = -1;
            for (int sm = 0; sm < 4; ++sm) {
                int w_s = -1;
                for (int w = sm; w < nw; w += 4)
                    if (used[w] < cap && (w_s < 0 || used[w] < used[w_s])) w_s = w;
                if (w_s >= 0 && (best < 0 || load[sm] < load[best])) { best = sm; bw = w_s; }
            }
            slot[(size_t)bw * cap + used[bw]] = c;
            ++used[bw];
            load[best] += cost[c];
        }
        return slot;
    }
    // one chunk per wave (the one-chunk instances, up to 16 waves): the exact assignment of the
    // chunks to the SIMDs' wave slots that minimises the largest SIMD total (LDPC_BS_DEAL=2).
    // LPT is not optimal where the SIMDs hold different numbers of waves: wman's 9 chunks
    // (3 + degree: 9 9 9 6 6 6 6 6 5) go 9 6 5 / 9 6 / 9 6 / 6 6 under LPT, a largest total of
    // 20 on the 3-wave SIMD (which also runs 3 of the 9 check waves), and 6 6 5 / 9 6 / 9 6 /
    // 9 6 exactly, 17.
    const int deal_mode = e ? atoi(e) : BS_DEAL_DEFAULT;
    if (deal_mode == 2 && cap == 1 && n <= nw && nw <= 16) {
        int slots[4] = {0, 0, 0, 0};
        for (int w = 0; w < nw; ++w) ++slots[w % 4];
        std::vector<int> cur(n, -1), best(n, -1);
        int load[4] = {0, 0, 0, 0}, used[4] = {0, 0, 0, 0};
        long long best_key = -1;
        // key: largest SIMD total, then the sum of squares (spread the rest)
        std::function<void(int)> rec = [&](int i) {
            const int mx = std::max(std::max(load[0], load[1]), std::max(load[2], load[3]));
            if (best_key >= 0 && (long long)mx * 1000000 > best_key) return;
            if (i == n) {
                const long long key = (long long)mx * 1000000 + (long long)load[0] * load[0] + (long long)load[1] * load[1] +
                                      (long long)load[2] * load[2] + (long long)load[3] * load[3];
                if (best_key < 0 || key < best_key) { best_key = key; best = cur; }
                return;
            }
            for (int sm = 0; sm < 4; ++sm) {
                if (used[sm] >= slots[sm]) continue;
                bool dup = false;                  // (a SIMD in the same state as one tried)
                for (int q = 0; q < sm; ++q)
                    if (used[q] < slots[q] && load[q] == load[sm] && slots[q] - used[q] == slots[sm] - used[sm]) dup = true;
                if (dup) continue;
                load[sm] += cost[order[i]];
                ++used[sm];
                cur[i] = sm;
                rec(i + 1);
                load[sm] -= cost[order[i]];
                --used[sm];
            }
        };
        rec(0);
        int next[4] = {0, 1, 2, 3};
        for (int i = 0; i < n; ++i) {                  // heaviest first: the SIMD's oldest wave
            const int sm = best[i];
            slot[(size_t)next[sm]] = order[i];
            next[sm] += 4;
        }
        return slot;
    }
    // virtual waves by LPT
    std::vector<std::vector<int>> vch(nw);
    std::vector<int> vload(nw, 0);
    for (int c : order) {
        int best = -1;
        for (int w = 0; w < nw; ++w)
            if ((int)vch[w].size() < cap &&
                (best < 0 || vload[w] < vload[best] || (vload[w] == vload[best] && vch[w].size() < vch[best].size())))
                best = w;
        vch[best].push_back(c);
        vload[best] += cost[c];
    }
    // virtual waves to physical ones: heaviest first to the SIMD with the smallest total
    std::vector<int> vorder(nw), sload(4, 0), next(4);
    for (int w = 0; w < nw; ++w) vorder[w] = w;
    std::stable_sort(vorder.begin(), vorder.end(), [&](int x, int y) { return vload[x] > vload[y]; });
    for (int sm = 0; sm < 4; ++sm) next[sm] = sm;
    for (int v : vorder) {
        int sm = -1;
        for (int q = 0; q < 4; ++q)
            if (next[q] < nw && (sm < 0 || sload[q] < sload[sm])) sm = q;
        const int w = next[sm];
        next[sm] += 4;
        sload[sm] += vload[v];
        for (size_t u = 0; u < vch[v].size(); ++u) slot[(size_t)w * cap + u] = vch[v][u];
    }
    return slot;
}

// dealing cost of each 64-lane check chunk (LPC lanes per check): the chunk's edge positions
// that hold a real edge for some lane (the kernels skip the rest wave-uniformly) plus the
// per-check work that does not depend on the degree
// check lane ql -> check cc | lane cj << 16 | lanes-per-check << 20 (-1: idle) of the uniform
// layout (checks in order, LPC lanes each)
std::vector<int32_t> uniform_lanes(const host::GraphTables& h, int LPC, int cn_lanes) {
    std::vector<int32_t> lanes((size_t)cn_lanes, -1);
    const int nc = h.M * h.z;
    for (int ql = 0; ql < cn_lanes; ++ql)
        if (ql / LPC < nc) lanes[(size_t)ql] = (ql / LPC) | ((ql % LPC) << 16) | (LPC << 20);
    return lanes;
}

// dealing cost of each 64-lane check chunk: 2 + the edge positions of its widest check
std::vector<int> check_chunk_cost_lanes(const host::GraphTables& h, const std::vector<int32_t>& lanes) {
    const int cch = (int)(lanes.size() / 64);
    std::vector<int> cost(cch, 2);
    for (int ch = 0; ch < cch; ++ch) {
        int pos = 0;
        for (int l = 0; l < 64; ++l) {
            const int32_t d = lanes[(size_t)64 * ch + l];
            if (d < 0) continue;
            const int i = (d & 0xFFFF) / h.z, L = (d >> 20) & 15;
            pos = std::max(pos, (h.row_ptr[i + 1] - h.row_ptr[i] + L - 1) / L);
        }
        cost[ch] += pos;
    }
    return cost;
}
std::vector<int> check_chunk_cost(const host::GraphTables& h, int LPC, int cch) {
    return check_chunk_cost_lanes(h, uniform_lanes(h, LPC, 64 * cch));
}

// Per-column rotation of a per-variable LDS array (bsc: Tv, 6 dwords per variable; bsl UCN: the
// hard decisions, 1 dword) read by the check lanes: variable (column j, index hh) is stored at
// j z + (hh + toff_j) mod z.  A half-wave of check lanes (32 / LPC consecutive checks, LPC edges
// each) reads, for edge position m, LPC runs of consecutive variables from LPC columns, which
// overlap mod 32 (the bank, for b32 reads and for b64 reads of 6-dword records alike) for most
// column pairs; a hill climb over the toff_j (the cost of a round: the most distinct indices on
// one bank, the sum of squared bank loads as the tie-break) spreads them.
std::vector<int> column_rotation_lanes(const host::GraphTables& h, int EPL, const std::vector<int32_t>& lanes) {
    const int z = h.z, cn_lanes = (int)lanes.size();
    std::vector<int> toff(h.N, 0);
    {
        std::vector<std::vector<std::pair<int, int>>> grp;          // (column, hh) per round
        std::vector<std::vector<int>> bycol(h.N);
        for (int h0 = 0; h0 < cn_lanes; h0 += 32)
            for (int m = 0; m < EPL; ++m) {
                std::vector<std::pair<int, int>> gl;
                for (int ql = h0; ql < h0 + 32 && ql < cn_lanes; ++ql) {
                    const int32_t d = lanes[(size_t)ql];
                    if (d < 0) continue;
                    const int cc = d & 0xFFFF, cj = (d >> 16) & 15, LPC = (d >> 20) & 15;
                    const int i = cc / z, hc = cc - i * z, kk = LPC * m + cj;
                    if (kk >= h.row_ptr[i + 1] - h.row_ptr[i]) continue;
                    const int pe = h.row_ptr[i] + kk;
                    gl.emplace_back(h.pe_col[pe], (hc + h.pe_shift[pe]) % z);
                }
                if (gl.empty()) continue;
                for (const auto& x : gl)
                    if (bycol[x.first].empty() || bycol[x.first].back() != (int)grp.size())
                        bycol[x.first].push_back((int)grp.size());
                grp.push_back(std::move(gl));
            }
        auto gcost = [&](const std::vector<std::pair<int, int>>& gl) {
            int cnt[32] = {0}, mx = 0, sq = 0;
            uint32_t seen[32];
            int ns = 0;
            for (const auto& x : gl) {
                const uint32_t t = (uint32_t)(x.first * z + (x.second + toff[x.first]) % z);
                bool dup = false;
                for (int q = 0; q < ns && !dup; ++q) dup = seen[q] == t;
                if (dup) continue;
                seen[ns++] = t;
                const int c = ++cnt[t & 31];
                mx = std::max(mx, c);
                sq += 2 * c - 1;
            }
            return mx * 4096 + sq;
        };
        std::vector<int> cost(grp.size());
        for (size_t gi = 0; gi < grp.size(); ++gi) cost[gi] = gcost(grp[gi]);
        uint64_t rng = 0x2545F4914F6CDD1Dull;
        for (int it = 0; it < 20000; ++it) {
            rng = rng * 6364136223846793005ull + 1442695040888963407ull;
            const int j = (int)((rng >> 33) % (uint64_t)h.N);
            if (bycol[j].empty()) continue;
            const int old = toff[j];
            toff[j] = (int)((rng >> 13) % (uint64_t)z);
            int before = 0, after = 0;
            std::vector<int> nc2(bycol[j].size());
            for (size_t q = 0; q < bycol[j].size(); ++q) {
                before += cost[bycol[j][q]];
                after += nc2[q] = gcost(grp[bycol[j][q]]);
            }
            if (after <= before) {
                for (size_t q = 0; q < bycol[j].size(); ++q) cost[bycol[j][q]] = nc2[q];
            } else {
                toff[j] = old;
            }
        }
    }
    return toff;
}
std::vector<int> column_rotation(const host::GraphTables& h, int LPC, int EPL, int cn_lanes) {
    return column_rotation_lanes(h, EPL, uniform_lanes(h, LPC, cn_lanes));
}

// first-generation start offsets of the one-workgroup-per-CU instances (BsArgs::stagger):
// LDPC_BS_STAGGER = the spread in microseconds (0: off)
void bs_stagger(bool one_per_cu, int* stagger, int* stagger_n) {
    *stagger = 0;
    *stagger_n = 0;
    const char* e = getenv("LDPC_BS_STAGGER");
    const double us = e ? atof(e) : (one_per_cu ? BS_STAGGER_US : 0.0);
    if (!(us > 0.0)) return;
    int dev = 0, ncu = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, dev) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    *stagger = (int)(us * 1e-3 * (double)khz / 512.0);      // s_sleep 8 = 512 clocks
    *stagger_n = ncu;
}

// the per-decode weight tables of both bit-sliced kernels (k_bs_tables)
int bs_make_tables(const Bufs& b, const DevGraph& g, int arows, int ar, int bcols, float step, int qmax,
                   float cu, bool ucn, FusedWorkspace& ws, uint32_t** alut, uint32_t** blut, hipStream_t s,
                   const int32_t** atid) {
    const size_t na = (size_t)b.T * ar * LUT_W, nb = (size_t)b.T * bcols * BLUT_W;
    const size_t bytes = (na + nb + (size_t)b.T * ar) * 4;     // + the alpha table ids
    if (bytes > ws.bs_lut_bytes) {
        if (ws.bs_lut) (void)hipFree(ws.bs_lut);
        ws.bs_lut = nullptr;
        ws.bs_lut_bytes = 0;
        ws.key_bslut[0] = ~0ull;
        if (hipMalloc(&ws.bs_lut, bytes) != hipSuccess) { (void)hipGetLastError(); return LDPC_ERR_OOM; }
        ws.bs_lut_bytes = bytes;
    }
    *alut = reinterpret_cast<uint32_t*>(ws.bs_lut);
    *blut = *alut + na;
    if (atid) *atid = reinterpret_cast<int32_t*>(*blut + nb);
    // (skipped when these tables are already in place: same weights, T and layout)
    const uint64_t kb[4] = {g.w_version, (uint64_t)b.T << 32 | (uint32_t)(arows << 16 | ar),
                            (uint64_t)__builtin_bit_cast(uint32_t, step) << 32 | __builtin_bit_cast(uint32_t, cu),
                            (uint64_t)qmax << 40 | (uint64_t)bcols << 1 | (ucn && b.alpha_ucn ? 1u : 0u)};
    if (std::equal(kb, kb + 4, ws.key_bslut)) return LDPC_OK;
    std::copy(kb, kb + 4, ws.key_bslut);
    const int ntab = b.T * (ar + bcols);
    // without UCN weights the alpha' slots (UCN instances) repeat the alpha tables (unused)
    const float* au = (ucn && b.alpha_ucn) ? b.alpha_ucn : b.alpha;
    hipLaunchKernelGGL(k_bs_tables, dim3((unsigned)((ntab + 127) / 128)), dim3(128), 0, s, b.alpha, au,
                       b.beta, g.row_ptr, b.T, g.E, g.N, arows, ar, bcols, step, 1.0f / step, qmax,
                       cu, *alut, *blut, reinterpret_cast<int32_t*>(*blut + nb));
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}
}  // namespace bs

// graph tables, built on the host (bs_graph_tables uploads them once per context)
struct BsHostTables {
    std::vector<uint32_t> vn;      // [VPL][64 nw][VNW]
    std::vector<int32_t> wdeg;     // [VPL][nw][3]
    std::vector<int32_t> cchunk;   // [nw][CPL]
    std::vector<uint32_t> chd;     // UCN: [cn_lanes][HDW]
};
static BsHostTables bs_host_tables(const DevGraph& g, const BsPlan& p) {
    const host::GraphTables& h = *g.host;
    const BsInst& k = kBsInst[p.inst];
    const int nv = g.n_vars, z = h.z;
    const int DV = k.DV, LPC = k.LPC;
    const int VNA = k.PK ? (DV + 1) / 2 : DV, VNW = VNA + 1;
    const int EPL = (k.D + LPC - 1) / LPC, HDW = (EPL + 1) / 2;
    const int nl = 64 * p.nw;
    std::vector<uint32_t> vn((size_t)k.VPL * nl * VNW, 0u);
    std::vector<int32_t> wdeg((size_t)3 * k.VPL * p.nw, 0);   // {most, fewest edges, column or -1}
    auto put = [&](uint32_t* w, int f, uint32_t addr) {
        if (k.PK) w[f >> 1] |= addr << (16 * (f & 1));
        else w[f] = addr;
    };
    auto slot_addr = [&](int i, int kk, int hc) {
        return p.off_slots + (uint32_t)(((size_t)p.lay[2 * i] + (size_t)(kk % LPC) * p.lay[2 * i + 1] +
                                         (size_t)(kk / LPC) * z + hc) * SLOT_B);
    };
    // variable lanes: variables by descending degree in chunks of 64; the chunks are dealt to
    // (wave, u) places so that the SIMDs get similar work (a chunk costs about 3 + dw units, dw
    // its largest degree); edge f of variable (col j, index hh) through proto edge pe (row i,
    // position kk) is slot (i, kk, (hh - shift) mod z)
    std::vector<int> order(nv);
    for (int v = 0; v < nv; ++v) order[v] = v;
    auto vdeg = [&](int v) { const int j = v / z; return h.col_ptr[j + 1] - h.col_ptr[j]; };
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return vdeg(x) > vdeg(y); });
    if (p.colalign) {               // each column's z variables, then 32 - z idle lanes (-1)
        std::vector<int> pad;
        for (int o = 0; o < nv; o += z) {
            pad.insert(pad.end(), order.begin() + o, order.begin() + o + z);
            pad.insert(pad.end(), (size_t)(32 - z), -1);
        }
        order.swap(pad);
    }
    const int nvo = (int)order.size();
    const int nch = (nvo + 63) / 64;
    std::vector<int> vcost(nch);
    for (int ch = 0; ch < nch; ++ch) vcost[ch] = 3 + vdeg(order[64 * ch]);
    const std::vector<int> vslot = deal_chunks(vcost, p.nw, k.VPL);
    for (int u = 0; u < k.VPL; ++u)
        for (int l = 0; l < nl; ++l) {
            uint32_t* q = &vn[((size_t)u * nl + l) * VNW];
            for (int f = 0; f < DV; ++f) put(q, f, p.off_zero);
            q[VNA] = 0xFFFFFFFFu;
        }
    // UCN instances: the hard decisions HD live at a per-column rotation of the variable index
    // (column_rotation: the check lanes' b32 reads of HD spread over the banks); a variable
    // lane's table word carries it as v | (HD index << 16)
    const char* ehd = getenv("LDPC_BS_HDPERM");
    const std::vector<int> hoff = (k.UCN && !(ehd && atoi(ehd) == 0))
                                      ? column_rotation(h, LPC, EPL, p.cn_lanes) : std::vector<int>(h.N, 0);
    auto hd_index = [&](int v) -> uint32_t {
        const int j = v / z, hh = v - j * z;
        return (uint32_t)(j * z + (hh + hoff[j]) % z);
    };
    const char* eo = getenv("LDPC_BS_VORDER");       // A/B: 0 keeps the graph's edge order
    const bool vorder = !(eo && atoi(eo) == 0);
    int vcost_before = 0, vcost_after = 0;
    std::vector<uint32_t> A((size_t)64 * DV);
    std::vector<int> dl(64);
    for (int w = 0; w < p.nw; ++w)
        for (int u = 0; u < k.VPL; ++u) {
            const int ch = vslot[(size_t)w * k.VPL + u];
            int dmax = 0, dmin = 1 << 30;
            if (ch < 0) {                 // no chunk at this place: the kernel skips it (dw < 0)
                wdeg[3 * ((size_t)u * p.nw + w)] = -1;
                wdeg[3 * ((size_t)u * p.nw + w) + 1] = 0;
                wdeg[3 * ((size_t)u * p.nw + w) + 2] = -1;
                continue;
            }
            int col = -2;                 // the chunk's column (-1: several)
            std::fill(A.begin(), A.end(), p.off_zero);
            std::fill(dl.begin(), dl.end(), 0);
            for (int l = 0; l < 64; ++l) {
                const int o = 64 * ch + l;
                if (o >= nvo || order[o] < 0) { dmin = 0; continue; }
                const int v = order[o], j = v / z, hh = v - j * z;
                col = (col == -2 || col == j) ? j : -1;
                const int c0 = h.col_ptr[j], dv = h.col_ptr[j + 1] - c0;
                for (int f = 0; f < dv; ++f) {
                    const int pe = h.col_pe[c0 + f], i = h.pe_row[pe];
                    int hc = hh - h.pe_shift[pe];
                    hc = hc < 0 ? hc + z : hc;
                    A[(size_t)l * DV + f] = slot_addr(i, pe - h.row_ptr[i], hc);
                }
                dl[l] = dv;
                dmax = std::max(dmax, dv);
                dmin = std::min(dmin, dv);
            }
            if (vorder) {
                const std::pair<int, int> c = host::order_variable_edges(A, dl, DV, std::min(DV, dmax));
                vcost_before += c.first;
                vcost_after += c.second;
            }
            for (int l = 0; l < 64; ++l) {
                const int o = 64 * ch + l;
                if (o >= nvo || order[o] < 0) continue;
                uint32_t* q = &vn[((size_t)u * nl + 64 * w + l) * VNW];
                for (int pw = 0; pw < VNA; ++pw) q[pw] = 0u;
                for (int f = 0; f < DV; ++f) put(q, f, A[(size_t)l * DV + f]);
                q[VNA] = k.UCN ? ((uint32_t)order[o] | (hd_index(order[o]) << 16)) : (uint32_t)order[o];
            }
            wdeg[3 * ((size_t)u * p.nw + w)] = dmax;
            wdeg[3 * ((size_t)u * p.nw + w) + 1] = dmin;
            wdeg[3 * ((size_t)u * p.nw + w) + 2] = col < 0 ? -1 : col;
        }
    if (getenv("LDPC_BS_VORDER_LOG"))
        fprintf(stderr, "bsl variable-phase bank cycles per slot word: %d -> %d\n", vcost_before, vcost_after);
    // check chunks (64 check lanes each) dealt to (wave, c) places; the small instances run
    // chunk w on wave w
    const int cch = p.cn_lanes / 64;
    std::vector<int32_t> cchunk((size_t)p.nw * k.CPL, -1);
    if (k.CPL == 1 && k.VPL == 1) {
        for (int w = 0; w < p.nw; ++w) cchunk[w] = w < cch ? w : -1;
    } else {
        const std::vector<int> cs = deal_chunks(check_chunk_cost(h, LPC, cch), p.nw, k.CPL);
        for (size_t x = 0; x < cs.size(); ++x) cchunk[x] = cs[x];
    }
    // UCN: per check lane, the LDS byte addresses (16-bit, packed) of its edges' hard decisions
    // HD[v] = 4 v (padding edges: the zero word)
    std::vector<uint32_t> chd;
    if (k.UCN) {
        chd.assign((size_t)p.cn_lanes * HDW, 0u);
        for (int ql = 0; ql < p.cn_lanes; ++ql) {
            const int cc = ql / LPC, cj = ql % LPC;
            for (int m = 0; m < EPL; ++m) {
                uint32_t addr = p.off_hdz;
                const int kk = LPC * m + cj;
                if (cc < g.n_checks) {
                    const int i = cc / z, hc = cc - i * z;
                    if (kk < h.row_ptr[i + 1] - h.row_ptr[i]) {
                        const int pe = h.row_ptr[i] + kk;
                        const int v = h.pe_col[pe] * z + (hc + h.pe_shift[pe]) % z;
                        addr = 4 * hd_index(v);
                    }
                }
                chd[(size_t)ql * HDW + (m >> 1)] |= addr << (16 * (m & 1));
            }
        }
    }
    BsHostTables t;
    t.vn.swap(vn);
    t.wdeg.swap(wdeg);
    t.cchunk.swap(cchunk);
    t.chd.swap(chd);
    return t;
}
static int bs_graph_tables(const DevGraph& g, const BsPlan& p, FusedWorkspace& ws, hipStream_t s) {
    if (ws.bs_graph) return LDPC_OK;
    BsHostTables t = bs_host_tables(g, p);
    const std::vector<uint32_t>& vn = t.vn;
    const std::vector<int32_t>& wdeg = t.wdeg;
    const std::vector<int32_t>& cchunk = t.cchunk;
    const std::vector<uint32_t>& chd = t.chd;
    const size_t nwords = vn.size() + wdeg.size() + p.lay.size() + cchunk.size() + chd.size();
    void* d = nullptr;
    if (hipMalloc(&d, nwords * 4) != hipSuccess) { (void)hipGetLastError(); return LDPC_ERR_OOM; }
    uint32_t* dp = reinterpret_cast<uint32_t*>(d);
    size_t at = 0;
    bool ok = true;
    auto up = [&](const void* src, size_t n) {
        if (n) ok = ok && hipMemcpyAsync(dp + at, src, n * 4, hipMemcpyHostToDevice, s) == hipSuccess;
        at += n;
    };
    up(vn.data(), vn.size());
    up(wdeg.data(), wdeg.size());
    up(p.lay.data(), p.lay.size());
    up(cchunk.data(), cchunk.size());
    up(chd.data(), chd.size());
    if (!ok || hipStreamSynchronize(s) != hipSuccess) {
        (void)hipFree(d);
        return LDPC_ERR_HIP;
    }
    ws.bs_graph = d;
    ws.bs_graph_inst = p.inst;
    return LDPC_OK;
}

bool bs_q8_ok(const DevGraph& g, int mode, bool ucn, float clip, int T, bool has_short) {
    const BsPlan p = bs_plan(g, mode, ucn, false, clip, T);
    if (!p.ok) return bsc_q8_ok(g, mode, ucn, clip, T, has_short);
    // (the in-prologue channel's tables borrow the slot region)
    return (!has_short || p.cu > 0.f) && (size_t)(p.off_pad - p.off_slots) >= sizeof(uint32_t) * AWGN_TAB_W;
}

int bs_decode(const DevGraph& g, const Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
              bool ucn, int64_t* counters, uint8_t* flags, uint32_t* bad, uint32_t* hdx, hipStream_t s) {
    const BsPlan p = bs_plan(g, mode, ucn, false, b.clip, b.T);
    if (!p.ok) return bsc_decode(g, b, ws, llr, mode, ucn, counters, flags, bad, hdx, s);
    if (ws.bs_graph && ws.bs_graph_inst != p.inst) {
        (void)hipFree(ws.bs_graph);
        ws.bs_graph = nullptr;
    }
    int st = bs_graph_tables(g, p, ws, s);
    if (st != LDPC_OK) return st;
    const BsInst& k = kBsInst[p.inst];
    const float step = mode_step_bs(mode);
    const int ar = (k.UCN ? 2 : 1) * p.arows;
    uint32_t *alut = nullptr, *blut = nullptr;
    const int32_t* atid = nullptr;
    st = bs_make_tables(b, g, p.arows, ar, p.bcols, step, bs_qmax(mode), p.cu, ucn, ws, &alut, &blut, s, &atid);
    if (st != LDPC_OK) return st;
    const int DV = k.DV;
    const int VNW = (k.PK ? (DV + 1) / 2 : DV) + 1;
    const uint32_t* gt = reinterpret_cast<const uint32_t*>(ws.bs_graph);
    BsArgs a{};
    a.llr = llr;
    if (b.q8) {                          // the in-prologue channel (ldpc_decode_awgn)
        const AwgnParams& g8 = *reinterpret_cast<const AwgnParams*>(b.gen8);
        a.gen.tab = b.q8;
        a.gen.k0 = g8.k0;
        a.gen.k1 = g8.k1;
        a.gen.offset = g8.offset;
        a.gen.nb = g8.nb;
        a.gen.kmin = g8.kmin;
        a.gen.ps = g8.ps;
        a.gen.pe = g8.pe;
        a.gen.ss = g8.ss;
        a.gen.se = g8.se;
        a.gen.lds = p.off_slots;
    }
    a.B = b.B;
    a.n_vars = g.n_vars;
    a.n_checks = g.n_checks;
    a.T = b.T;
    a.target_bits = b.target_bits;
    a.cn_lanes = p.cn_lanes;
    a.cn_dmin = p.cn_dmin;
    a.inv = 1.0f / step;
    a.cu = p.cu > 0.f ? p.cu : -1.f;
    a.qmax = bs_qmax(mode);
    a.ucn = p.ucn ? 1 : 0;
    a.ucn_iter = g.w_ucn_iter;
    a.beta_id = g.w_beta_id_mask;        // (identity on m <= 15 implies it on m <= qmax)
    a.row_ptr = g.row_ptr;
    a.z = g.z;
    a.vn_tab = gt;
    const size_t nvt = (size_t)k.VPL * 64 * p.nw * VNW;
    a.vn_wdeg = reinterpret_cast<const int32_t*>(gt + nvt);
    a.row_lay = a.vn_wdeg + 3 * (size_t)k.VPL * p.nw;
    a.cn_chunk = a.row_lay + 2 * (size_t)g.M;
    a.cn_hd = reinterpret_cast<const uint32_t*>(a.cn_chunk + (size_t)p.nw * k.CPL);
    a.alut = alut;
    a.blut = blut;
    a.arows = p.arows;
    a.bcols = p.bcols;
    // the fixed-set channel tables cover the grids whose magnitudes saturate at 15 (q = 5, -5)
    a.btid = (bs_qmax(mode) == QMAX && !getenv("LDPC_BS_NOBFIX")) ? g.beta_tid : nullptr;
    a.btid_n = g.N;
    a.atid = getenv("LDPC_BS_NOAFIX") ? nullptr : atid;
    a.counters = counters;
    a.flags = flags;
    a.bad = bad;
    a.iter_wrong = b.iter_wrong;
    a.hdx = hdx;
    bs_stagger(k.VPL > 1 || k.CPL > 1, &a.stagger, &a.stagger_n);
    a.off_slots = p.off_slots;
    a.off_pad = p.off_pad;
    a.off_zero = p.off_zero;
    a.off_red = p.off_red;
    a.off_alut = p.off_alut;
    a.off_blut = p.off_blut;
    a.off_hdz = p.off_hdz;
    a.off_btid = p.off_btid;
    a.off_hdl = p.off_hdl;
    a.off_preb = p.off_preb;
    a.off_ch = p.off_ch;
    if (const char* e = getenv("LDPC_DIAG_ABLATE")) a.ablate = atoi(e);   // -DBS_DIAG builds
    const int nblocks = (int)((b.B + PACK - 1) / PACK);
    static const auto kLaunch = launch_table(std::make_integer_sequence<int, kBsNInst>{});
    // (A/B: LDPC_BS_LDS_MIN=bytes requests at least that much dynamic LDS per workgroup, fewer
    // workgroups per CU -- the occupancy experiment; the kernel uses only its own layout)
    static const size_t lds_min = [] { const char* e = getenv("LDPC_BS_LDS_MIN"); return e ? (size_t)atol(e) : 0; }();
    const size_t lds = std::min(std::max(p.lds, lds_min), (size_t)BS_LDS_MAX);
#ifdef BS_STAMP
    // diagnostic build: per-wave phase clocks of this decode, printed to stderr
    static unsigned long long* dst = nullptr;
    if (!dst && hipMalloc(reinterpret_cast<void**>(&dst), 256 * 8) != hipSuccess) return LDPC_ERR_OOM;
    if (hipMemsetAsync(dst, 0, 256 * 8, s) != hipSuccess) return LDPC_ERR_HIP;
    a.stamps = dst;
    st = kLaunch[p.inst](a, nblocks, p.nw, lds, s, b.q8 != nullptr);
    unsigned long long hst[256];
    if (st != LDPC_OK || hipMemcpyAsync(hst, dst, sizeof(hst), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return st != LDPC_OK ? st : LDPC_ERR_HIP;
    fprintf(stderr, "bs_stamp inst %d T %d q8 %d: per pack, shader clocks [check, check-barrier, var, var-barrier | "
            "entry, channel, ch-barrier, tables, first-var, check-setup | epilogue]\n", p.inst, b.T, b.q8 != nullptr);
    static const int order[] = {0, 1, 2, 3, 8, 9, 10, 11, 12, 4, 5};
    for (int w = 0; w < p.nw && w < 16; ++w) {
        const double n = (double)(hst[16 * w + 15] ? hst[16 * w + 15] : 1);
        fprintf(stderr, "  wave %2d:", w);
        for (const int i : order) fprintf(stderr, " %8.0f", hst[16 * w + i] / n);
        fprintf(stderr, "  | SIMD %5.3f %5.3f %5.3f %5.3f\n", (hst[16 * w + 13] & 0xFFFFFFFFull) / n,
                (hst[16 * w + 13] >> 32) / n, (hst[16 * w + 14] & 0xFFFFFFFFull) / n, (hst[16 * w + 14] >> 32) / n);
    }
    return st;
#else
    return kLaunch[p.inst](a, nblocks, p.nw, lds, s, b.q8 != nullptr);
#endif
}

}  // namespace ldpc

// ---- host-side bounds check of the bit-sliced kernel's reads (test infrastructure) -----------
// For a plan and its host tables (the launch's own planning code: plan_inst, bs_host_tables),
// every index k_bs reads is recomputed on the host -- the kernel's predicates restated from
// ldpc_bs_kernel.h -- and checked against what the context allocates: the global tables
// (vn_tab, vn_wdeg, row_ptr, row_lay, cn_chunk, cn_hd, the channel-table ids), the LDS regions
// (slots, PAD / ZERO, HD, RED, the alpha / beta tables, the per-lane words) and the dynamic LDS
// size.  The r4c fault (a one-chunk UCN instance read cn_hd for the waves past cn_lanes) is the
// class it guards: LDPC_BOUNDS_PRE_GUARD drops the `ql < cn_lanes` term of that read, as the
// kernel had it before the fix, so a test can see the check catch it.
namespace ldpc {
namespace bs {
enum { LDPC_BOUNDS_PRE_GUARD = 1 };
struct BoundsReport {
    int violations = 0;
    std::string first;
    void fail(const char* what, long long idx, long long lim) {
        if (violations++ == 0) {
            char buf[160];
            snprintf(buf, sizeof(buf), "%s: index %lld outside [0, %lld)", what, idx, lim);
            first = buf;
        }
    }
    void in(const char* what, long long idx, long long lim) {
        if (idx < 0 || idx >= lim) fail(what, idx, lim);
    }
    // an LDS byte range [a, a + n) inside [lo, hi)
    void lds(const char* what, long long a, long long n, long long lo, long long hi) {
        if (a < lo || a + n > hi) fail(what, a, hi);
    }
};

static int bs_bounds_check(const DevGraph& g, const BsPlan& p, const BsHostTables& t, int T, int flags,
                           BoundsReport& r) {
    const BsInst& k = kBsInst[p.inst];
    const host::GraphTables& h = *g.host;
    const int LPC = k.LPC, VPL = k.VPL, CPL = k.CPL, DV = k.DV;
    const int EPL = (k.D + LPC - 1) / LPC, HDW = (EPL + 1) / 2, OB = 4 / LPC;
    const int VNA = k.PK ? (DV + 1) / 2 : DV, VNW = VNA + 1;
    const int NT = 64 * p.nw, nwv = p.nw, nv = g.n_vars, z = h.z;
    const bool UCN = k.UCN, ucn = UCN && p.ucn;
    const int AR = UCN ? 2 * p.arows : p.arows;
    const long long AL = (long long)AR * LUT_W, BL = (long long)p.bcols * BLUT_W;
    const long long lds = (long long)p.lds;
    const bool SKIPM = CPL > 1;
    const bool GBL = BS_GBLDS && CPL == 1 && !BS_CH_LDS;
    const bool HDL = BS_HDLDS && UCN && CPL == 1;
    // (ALDS: GW words per lane, the slot base and then the packed slot addresses)
    const int HWA = (EPL + 1) / 2;
    const int GW = (GBL && k.PK && BS_ALDS) ? ((1 + HWA) | 1) : 1;
    // the allocations
    if (getenv("LDPC_BOUNDS_VERBOSE"))
        fprintf(stderr, "bs plan: inst %d nw %d ucn %d lds %lld (slots %u..%u, alut %u, blut %u, ch %u, hdl %u)\n",
                p.inst, p.nw, (int)p.ucn, lds, p.off_slots, p.off_pad, p.off_alut, p.off_blut, p.off_ch, p.off_hdl);
    r.in("lds size", lds, (long long)BS_LDS_MAX + 1);
    if ((long long)t.vn.size() != (long long)VPL * NT * VNW) r.fail("vn_tab size", (long long)t.vn.size(), (long long)VPL * NT * VNW);
    r.lds("RED", p.off_red, 4LL * (16 + ((T + 3) & ~3) + BS_FLORW), 0, p.off_alut);
    r.lds("ALUT", p.off_alut, 4 * 2 * AL, 0, p.off_blut);
    r.lds("BLUT", p.off_blut, 4 * 2 * BL, 0, lds);
    r.lds("PAD+ZERO", p.off_pad, 2 * SLOT_B, p.off_slots, p.off_red);
    // (PREB) the check-idle waves' lanes, 16 B each
    if (p.off_preb)
        for (int w = p.cn_lanes / 64; w < nwv; ++w)
            r.lds("PREB", p.off_preb + 16LL * (64 * w - p.cn_lanes), 16LL * 64, p.off_preb, lds);
    if (UCN) r.lds("HD", 0, 4LL * (nv + 1), 0, p.off_slots);
    // the in-prologue channel's sampler tables (Q8 builds, gen.lds = off_slots): inside the slot
    // region, which the kernel writes only after the prologue, and clear of PAD / ZERO / RED /
    // the tables the prologue writes -- whenever bs_q8_ok lets the Q8 build run on this plan
    if ((size_t)(p.off_pad - p.off_slots) >= sizeof(uint32_t) * AWGN_TAB_W)
        r.lds("channel tables", p.off_slots, 4LL * AWGN_TAB_W, p.off_slots, p.off_pad);
    // ---- variable phase: per (u, lane)
    for (int u = 0; u < VPL; ++u)
        for (int w = 0; w < nwv; ++w) {
            const long long wi = 3LL * (u * nwv + w);
            r.in("vn_wdeg", wi + 2, (long long)t.wdeg.size());
            if (wi + 2 >= (long long)t.wdeg.size()) continue;
            const int dw = t.wdeg[(size_t)wi], pcol = t.wdeg[(size_t)wi + 2];
            if (pcol >= 0) r.in("btid column", pcol, h.N);
            // channel-table ids: the variable phase of iteration t reads btid[(t + 1) N + col]
            // for t + 1 < T (col = 0 with one column table), and beta_tid holds [T_w][N] rows,
            // T <= T_w by host::check_decode
            if (dw >= 0 && T > 1) {
                const long long col = p.bcols == 1 ? 0 : pcol;
                if (col >= 0) r.in("btid", (long long)(T - 1) * h.N + col, (long long)T * h.N);
            }
            for (int l = 0; l < 64; ++l) {
                const long long ti = ((long long)u * NT + 64LL * w + l) * VNW;
                r.in("vn_tab", ti + VNA, (long long)t.vn.size());
                if (ti + VNA >= (long long)t.vn.size()) continue;
                const uint32_t* q = &t.vn[(size_t)ti];
                const int vv = (int)q[VNA];
                const int v = (UCN && vv >= 0) ? (vv & 0xFFFF) : vv;
                if (v >= nv) r.fail("variable", v, nv);
                if (vv >= 0 && UCN) r.in("HD index", (long long)((uint32_t)vv >> 16), nv);
                if (vv >= 0 && p.bcols > 1) r.in("beta table", v / (nv / p.bcols), p.bcols);
                for (int f = 0; f < DV && f < dw; ++f) {     // the kernel reads f < dw (wave max)
                    const uint32_t a = k.PK ? ((f & 1) ? (q[f >> 1] >> 16) : (q[f >> 1] & 0xFFFFu)) : q[f];
                    if (a != p.off_zero) r.lds("variable slot", a, SLOT_B, p.off_slots, p.off_pad);
                }
            }
        }
    // ---- check phase: per (wave, chunk, lane)
    for (int w = 0; w < nwv; ++w)
        for (int c = 0; c < CPL; ++c) {
            r.in("cn_chunk", (long long)w * CPL + c, (long long)t.cchunk.size());
            const int gchunk = CPL == 1 ? w : t.cchunk[(size_t)w * CPL + c];
            const bool active = CPL == 1 ? w * 64 < p.cn_lanes : gchunk >= 0;
            int gm = EPL;
            if (SKIPM) {                                   // the chunk's real positions (wave_or)
                uint32_t any = 0u;
                for (int l = 0; l < 64; ++l) {
                    const int ql = std::max(gchunk, 0) * 64 + l, cc = ql / LPC;
                    const int ci = std::min(cc / z, g.n_checks / z - 1);
                    const int gdeg = cc < g.n_checks ? h.row_ptr[ci + 1] - h.row_ptr[ci] : 0;
                    any |= (1u << ((gdeg + LPC - 1) / LPC)) - 1u;
                }
                gm = __builtin_popcount(any);
                // the kernels' switch over the real positions covers 1 .. EPL (BS_MIN2_CASE)
                if (active) r.in("real positions - 1 (the min2 switch)", gm - 1, EPL);
            }
            for (int l = 0; l < 64; ++l) {
                const int ql = std::max(gchunk, 0) * 64 + l, cc = ql / LPC, cj = l % LPC;
                const int ci = std::min(cc / z, g.n_checks / z - 1);
                r.in("row_ptr", ci + 1, h.M + 1);
                r.in("row_lay", 2LL * ci + 1, (long long)p.lay.size());
                const int gdeg = cc < g.n_checks ? h.row_ptr[ci + 1] - h.row_ptr[ci] : 0;
                // the lane's tables (read by every lane of a chunk, active or not)
                if (UCN) {
                    const bool guard = (flags & LDPC_BOUNDS_PRE_GUARD) ? true : ql < p.cn_lanes;
                    if (ucn && gchunk >= 0 && guard)
                        for (int pp = 0; pp < HDW; ++pp) r.in("cn_hd", (long long)ql * HDW + pp, (long long)t.chd.size());
                }
                if (GBL) r.lds("per-lane words", p.off_ch + 4LL * GW * (64 * w + l), 4LL * GW, p.off_ch, lds);
                if (HDL)
                    for (int pp = 0; pp < HDW; ++pp) r.lds("HD addresses", p.off_hdl + 4LL * (pp * NT + 64 * w + l), 4, p.off_hdl, lds);
                if (!active) continue;
                const long long gbase = p.off_slots +
                    ((long long)p.lay[2 * ci] + (long long)cj * p.lay[2 * ci + 1] + (cc - ci * z)) * SLOT_B;
                for (int m = 0; m < EPL; ++m) {
                    if (SKIPM && m >= gm) continue;
                    const bool re = LPC * m + LPC - 1 < p.cn_dmin || LPC * m + cj < gdeg;
                    const long long a = re ? gbase + (long long)m * z * SLOT_B : p.off_pad;
                    r.lds("check slot", a, SLOT_B, p.off_slots, p.off_red);
                    if (re && a + SLOT_B > p.off_pad) r.fail("check slot past the slot region", a, p.off_pad);
                    if (ucn && cc < g.n_checks && ql < p.cn_lanes && (size_t)ql * HDW + (m >> 1) < t.chd.size()) {
                        const uint32_t hw = t.chd[(size_t)ql * HDW + (m >> 1)];
                        const uint32_t ha = (m & 1) ? (hw >> 16) : (hw & 0xFFFFu);
                        r.lds("HD read", ha, 4, 0, (long long)p.off_hdz + 4);
                    }
                }
                // the alpha tables: lane cj evaluates OB bits of the row's table (and alpha')
                const long long ctab = p.off_alut + (long long)(p.arows > 1 ? ci : 0) * LUT_W * 4 + (long long)cj * OB * 64;
                const long long last = ctab + 4LL * AL + (UCN ? (long long)p.arows * LUT_W * 4 : 0) + (OB - 1) * 64 + 3 * 16;
                r.lds("alpha table", ctab, 16, p.off_alut, p.off_alut + 4 * 2 * AL);
                r.lds("alpha table (odd t, alpha')", last, 16, p.off_alut, p.off_alut + 4 * 2 * AL);
            }
        }
    return r.violations;
}
}  // namespace bs
}  // namespace ldpc

// One plan per (instance, UCN) that fits a proto graph with the given weight properties, each
// checked by bs_bounds_check.  Returns the number of plans checked (>= 0) and writes the first
// violation into msg ("" when none); *violations = the total.  Host only: no device is touched.
extern "C" int ldpc_debug_bs_bounds(const int32_t* proto, int32_t M, int32_t N, int32_t z, int32_t T,
                                    int32_t mode, int32_t alpha_uniform, int32_t beta_uniform,
                                    float clip, int32_t flags, int32_t* violations, char* msg,
                                    int32_t msg_len) {
    using namespace ldpc;
    using namespace ldpc::bs;
    if (!proto || !violations || T <= 0) return LDPC_ERR_ARG;
    host::GraphTables h;
    const int st = host::build_graph(proto, M, N, z, h);
    if (st != LDPC_OK) return st;
    DevGraph g{};
    g.M = h.M; g.N = h.N; g.z = h.z; g.E = h.E;
    g.n_checks = h.M * h.z; g.n_vars = h.N * h.z; g.n_edges = h.E * h.z; g.max_cdeg = h.max_cdeg;
    g.h_row_ptr = h.row_ptr.data();
    g.host = &h;
    g.w_alpha_uniform = alpha_uniform;
    g.w_alpha_pair_uniform = alpha_uniform;
    g.w_beta_uniform = beta_uniform;
    g.w_beta_nonneg = 1;
    int min_cdeg = 1 << 30;
    for (int i = 0; i < h.M; ++i) min_cdeg = std::min(min_cdeg, h.row_ptr[i + 1] - h.row_ptr[i]);
    int checked = 0;
    *violations = 0;
    std::string first;
    for (int i = 0; i < kBsNInst; ++i)
        for (int u = 0; u < 2; ++u) {
            const BsPlan p = plan_inst(g, i, u != 0, clip, min_cdeg, mode, T);
            if (!p.ok) continue;
            const BsHostTables t = bs_host_tables(g, p);
            BoundsReport r;
            bs_bounds_check(g, p, t, T, flags, r);
            ++checked;
            if (r.violations && first.empty()) {
                char buf[64];
                snprintf(buf, sizeof(buf), "instance %d%s: ", i, u ? " ucn" : "");
                first = std::string(buf) + r.first;
            }
            *violations += r.violations;
        }
    // the compressed kernel (bsc, no UCN): its plan with and without the beta = 1 build's
    // mixed-lane instances
    for (int b1 = 0; b1 < 2; ++b1) {
        if (b1 && !beta_uniform) continue;
        g.w_beta_one = b1;
        BoundsReport r;
        const int n = bsc_debug_bounds(g, mode, clip, T, r.violations, r.first);
        if (n <= 0) continue;
        ++checked;
        if (r.violations && first.empty()) first = std::string(b1 ? "bsc beta=1: " : "bsc: ") + r.first;
        *violations += r.violations;
    }
    if (msg && msg_len > 0) {
        std::strncpy(msg, first.c_str(), (size_t)msg_len - 1);
        msg[msg_len - 1] = 0;
    }
    return checked;
}
