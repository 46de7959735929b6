// rq_gen.h -- one source's arrival stream as a step machine (one lane, one source).
//
// Shared by rq_gen_streams (streams written to HBM) and the fused sweep (rings
// refilled in LDS), so both produce the same bits.  One step() = one candidate:
//   Poisson / Poisson2  opt_model.py:424-433 / :396-405 -- exponential gaps
//                       t += Exp(1) / rate (one draw per arrival)
//   Hawkes              opt_model.py:466-490 -- Ogata thinning with the exponential
//                       kernel's O(1) recurrence for lambda; two draws (Exp, uniform)
//                       per candidate; accept when U * B < lambda (the reference's
//                       U < lambda / B, division-free).  The bound B starts at lambda
//                       at the last accepted arrival and, after a rejection, is
//                       refreshed to lambda at the rejected candidate (lambda only
//                       decays until the next arrival, so it still bounds it).  The
//                       reference keeps the stale bound: the same point process (law),
//                       a different draw sequence and more candidates per arrival.
//   PiecewiseConst      opt_model.py:642-663 -- thinning of exponential gaps at the
//                       max rate; two draws per candidate
//   RealData            opt_model.py:722-750 -- the given (host-filtered) times
// Draw d of a stream is half d&1 of Philox4x32-10 call d>>1 under key (seed, salt):
// the first half of a call is only taken with d even, so every candidate of a
// two-draw kind is exactly one call.
#pragma once
#include "rq_device.h"
#include "rq_internal.h"

namespace rq {

struct SrcGen {
    uint32_t k0, k1;        // Philox key (seed, kind salt)
    uint32_t d;             // next draw index (< 2^32 draws per source)
    // the draws are turned into exponentials ahead of their use, so the Philox rounds and
    // the logarithm run beside the dependent chain of the candidate before (the generator
    // is latency-bound, not issue-bound): Poisson takes both halves of a call at its even
    // draw (en: the odd draw's exponential); Hawkes / PiecewiseConst (one call per
    // candidate) hold the next candidate's exponential and acceptance uniform (e1n, u2n)
    double en, e1n, u2n;
    int kind;
    bool done;
    double t;               // candidate base time
    double tau, eta, B;     // Hawkes: last accepted time, excitation at tau, bound
    double inv;             // 1 / rate (Poisson), 1 / max rate (PWConst), 1 / B (Hawkes)
    double p0, p1, nbeta;   // rate | (l_0, alpha, -beta)
    const uint64_t* etab;   // rq_exp's table (RQ_EXP_TAB_INIT): LDS or __constant__ copy
    const double* ta;       // PWConst change times / RealData times
    const double* tb;       // PWConst rates
    int na, ri;

    __device__ __forceinline__ void none()
    {
        etab = nullptr;
        kind = RQ_SRC_NONE;
        done = true;
        d = 0u;
        en = e1n = u2n = 0.0;
    }
    // Philox call `call` of this stream -> the exponential of its first half and the
    // uniform of its second
    __device__ __forceinline__ void draw2(uint32_t call, double& e, double& u) const
    {
        uint32_t c[4] = {call, 0u, 0u, 0u};
        philox4x32_10(c, k0, k1);
        e = rq_std_exponential(rq_uniform53(c[0], c[1]));
        u = rq_uniform53(c[2], c[3]);
    }

    __device__ __forceinline__ void init(const GenArgs& a, int j, int64_t i, const uint64_t* etab_)
    {
        etab = etab_;
        const bool is_ctrl = j == a.ctrl_idx;
        kind = is_ctrl ? a.ctrl_stream_kind : a.kind[j];
        const int64_t k = a.seed_mod > 0 ? i % a.seed_mod : i;
        uint32_t seed;
        if (is_ctrl) {
            seed = a.ctrl_seed ? a.ctrl_seed[i] : a.ctrl_seed0 + (uint32_t)k;
        } else if (a.randomize) {
            const uint32_t u = a.world_seed ? a.world_seed[i] : a.world_seed0 + (uint32_t)k;
            seed = u + 99u * (uint32_t)a.orig_idx[j];   // randomize_other_sources, opt_model.py:795-804
        } else {
            seed = a.seed[j];
        }
        k0 = seed;
        k1 = kind_salt(kind, is_ctrl);
        d = 0u;
        en = e1n = u2n = 0.0;
        done = false;
        t = a.start;
        tau = a.start;
        eta = 0.0;
        B = 0.0;
        inv = 0.0;
        p0 = p1 = nbeta = 0.0;
        ta = tb = nullptr;
        na = ri = 0;
        if (kind == RQ_SRC_POISSON || kind == RQ_SRC_POISSON2) {
            const double rate = is_ctrl ? a.ctrl_rate[i] : a.p0[j];
            if (rate > 0.0) inv = 1.0 / rate;
            else done = true;
        } else if (kind == RQ_SRC_HAWKES) {
            p0 = a.p0[j];
            p1 = a.p1[j];
            nbeta = -a.p2[j];
            B = p0;   // lambda at start (no excitation yet)
            if (B > 0.0) inv = 1.0 / B;
            else done = true;
        } else if (kind == RQ_SRC_PWCONST) {
            na = a.arr_n[j];
            ta = a.arr_a + a.arr_off[j];
            tb = a.arr_b + a.arr_off[j];
            double mx = tb[0];
            for (int q = 1; q < na; ++q) mx = tb[q] > mx ? tb[q] : mx;
            if (mx > 0.0) inv = 1.0 / mx;
            else done = true;
            p0 = mx;
        } else if (kind == RQ_SRC_REALDATA) {
            const int rk = (a.rd_k && !is_ctrl) ? a.rd_k[j] : -1;
            if (rk >= 0) {   // this replica's own times (a registered static broadcaster)
                const int64_t o = a.rd_off[i * a.n_rd + rk];
                na = (int)(a.rd_off[i * a.n_rd + rk + 1] - o);
                ta = a.rd_times + o;
            } else {
                na = a.arr_n[j];
                ta = a.arr_a + a.arr_off[j];
            }
            done = na <= 0;
        } else {
            done = true;   // the controlled slot of an Opt / wall-only run: no stream
        }
        if (!done && (kind == RQ_SRC_HAWKES || kind == RQ_SRC_PWCONST)) draw2(0u, e1n, u2n);
    }

    // one candidate; true (and *out) when it is an arrival.  Sets done past `end`.
    __device__ __forceinline__ bool step(double* out, double end)
    {
        if (done) return false;
        if (kind == RQ_SRC_REALDATA) {
            *out = ta[ri];
            ++ri;
            done = ri >= na;
            return true;
        }
        const bool poisson = kind == RQ_SRC_POISSON || kind == RQ_SRC_POISSON2;
        double e, u2 = 0.0;
        if (poisson) {
            if ((d & 1u) == 0u) {
                uint32_t c[4] = {d >> 1, 0u, 0u, 0u};
                philox4x32_10(c, k0, k1);
                e = rq_std_exponential(rq_uniform53(c[0], c[1]));
                en = rq_std_exponential(rq_uniform53(c[2], c[3]));
            } else {
                e = en;
            }
            d += 1u;
        } else {
            // two draws per candidate (d even): this candidate's came one call ahead
            e = e1n;
            u2 = u2n;
            d += 2u;
            draw2(d >> 1, e1n, u2n);
        }
        const double tc = t + e * inv;
        if (!(tc <= end)) {
            done = true;
            return false;
        }
        t = tc;
        if (poisson) {
            *out = tc;
            return true;
        }
        if (kind == RQ_SRC_HAWKES) {
            const double decay = rq_exp_t(nbeta * (tc - tau), etab);
            const double rate = p0 + eta * decay;
            const bool acc = u2 * B < rate;   // u2 < rate / B without the f64 division
            // accepted: the next candidate starts at tc under B = lambda just after it;
            // rejected: lambda only decays until the next arrival, so lambda(tc) bounds it
            // from here on -- thinning continues at the refreshed (lower) bound.  One
            // division on the merged path (the two branches diverge within a wave).
            if (acc) {
                eta = eta * decay + p1;
                tau = tc;
                B = p0 + eta;
            } else {
                B = rate;
            }
            if (B > 0.0) inv = 1.0 / B;
            else done = true;   // lambda == 0 from here on: no further arrival
            if (acc) *out = tc;
            return acc;
        }
        // PiecewiseConst: rate(t) = rates[bisect_right(change_times, t) - 1]
        int lo = 0, hi = na;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (tc < ta[mid]) hi = mid;
            else lo = mid + 1;
        }
        int idx = lo - 1;
        if (idx < 0) idx += na;
        if (u2 * p0 < tb[idx]) {
            *out = tc;
            return true;
        }
        return false;
    }
};

}  // namespace rq
