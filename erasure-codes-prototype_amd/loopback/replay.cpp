// libecg_replay.so: the proxies' per-stripe repair and merge call sequences, issued from C++ as the proxies
// issue them, for bench.py (config 3 `--workload lrc-repair`, config 4 `--workload pc-merge`, and the line's
// config3 / config4 objects).
//
// The reference's main/help repair with partial decoding makes, per stripe, three ErasureCode calls
// (handle_repair.cpp:249,371-376,566): a helper proxy's encode_partial_blocks_for_decoding over its
// partition's survivors, the main proxy's own encode_partial_blocks_for_decoding, and perform_addition of
// the two partials into the repaired block.  Driving those calls one by one from Python would measure
// the interpreter (~10 us per call), not the engine; the proxy is C++.  So this replays the same calls
// through the C ABI (include/ecg.h, nothing else), on HBM blocks, in one of three forms:
//   0 direct   every call launched on its own;
//   1 scope    calls recorded in deferred-batch scopes of `scope_stripes` stripes (ecg_batch_begin/end);
//   2 scratch  the same scopes with the partial buffers declared scratch (ecg_batch_scratch): the three
//              calls of a repair compose into one region product and the partials never reach HBM.
// Not part of libecg (the product); a caller of it, like loopback/.
#include <thread>
#include <vector>

#include "../../include/ecg.h"

extern "C" {

// Repairs launch stripes i < S: stripe st = stripe_of[i] (host int[S]) of the strided batch (block b at
// base + st * sstride + b * bstride) loses block fail[p], p = pattern_of[i] (host int[S]); pattern p's
// n_surv survivors surv[p * n_surv ..], of which the helper partition holds help[p * n_help ..] and the
// main proxy main_[p * n_main ..].  Partials of launch stripe i at partials + (2 i + j) * B (j = 0 helper,
// 1 main); the repaired block of stripe st at out + st * out_stride.  Asynchronous on `stream`; returns 0 or the first
// negative ecg_* status.
int ecg_replay_partial_repair(ecg_ec* ec, int form, int scope_stripes, char* base, long long sstride,
                              long long bstride, int B, int S, const int* stripe_of, const int* pattern_of,
                              const int* fail, int n_surv, const int* surv, int n_help, const int* help, int n_main,
                              const int* main_, char* partials, char* out, long long out_stride, void* stream) {
    if (!ec || form < 0 || form > 2 || B <= 0 || S < 0 || n_help < 1 || n_main < 1 || n_surv < 1 ||
        (form > 0 && scope_stripes < 1))
        return ECG_EINVAL;
    int rc = ecg_ec_set_memory(ec, ECG_MEM_DEVICE, stream);
    if (rc) return rc;
    std::vector<char*> hp(n_help), mp(n_main);
    auto repair = [&](int i) -> int {
        const int st = stripe_of[i], p = pattern_of[i];
        char* blk0 = base + (long long)st * sstride;
        for (int j = 0; j < n_help; j++) hp[j] = blk0 + (long long)help[p * n_help + j] * bstride;
        for (int j = 0; j < n_main; j++) mp[j] = blk0 + (long long)main_[p * n_main + j] * bstride;
        char* pp[2] = {partials + (2LL * i) * B, partials + (2LL * i + 1) * B};
        const int* sv = surv + (long long)p * n_surv;
        // help_repair (handle_repair.cpp:566-567), then the main proxy's own partial (:249)
        int r = ecg_ec_encode_partial_blocks_for_decoding(ec, hp.data(), &pp[0], B, help + p * n_help, n_help, sv,
                                                          n_surv, fail + p, 1);
        if (r) return r;
        r = ecg_ec_encode_partial_blocks_for_decoding(ec, mp.data(), &pp[1], B, main_ + p * n_main, n_main, sv, n_surv,
                                                      fail + p, 1);
        if (r) return r;
        char* o = out + (long long)st * out_stride;
        return ecg_ec_perform_addition(ec, pp, &o, B, 2, 1);  // handle_repair.cpp:371-376
    };
    if (form == 0) {
        for (int i = 0; i < S; i++)
            if ((rc = repair(i))) return rc;
        return 0;
    }
    for (int c0 = 0; c0 < S; c0 += scope_stripes) {
        const int c1 = c0 + scope_stripes < S ? c0 + scope_stripes : S;
        if ((rc = ecg_batch_begin())) return rc;
        if (form == 2 && (rc = ecg_batch_scratch(partials + 2LL * c0 * B, (size_t)(c1 - c0) * 2 * B))) {
            ecg_batch_end();
            return rc;
        }
        for (int i = c0; i < c1 && !rc; i++) rc = repair(i);
        const int re = ecg_batch_end();
        if (rc) return rc;
        if (re) return re;
    }
    return 0;
}

// The same per-call sequence issued CONCURRENTLY, as the proxy issues it: the reference runs every request
// on its own detached thread (proxy.cpp:416-419; handle_repair.cpp:246-252,370-376 per repair).  Thread t
// takes the contiguous share [t S / n, (t + 1) S / n) of the repairs with its own ErasureCode handle ecs[t]
// and its own stream streams[t]; threads are joined before returning (their launches stay asynchronous).
int ecg_replay_partial_repair_mt(ecg_ec** ecs, void** streams, int nthreads, int form, int scope_stripes, char* base,
                                 long long sstride, long long bstride, int B, int S, const int* stripe_of,
                                 const int* pattern_of, const int* fail, int n_surv, const int* surv, int n_help,
                                 const int* help, int n_main, const int* main_, char* partials, char* out,
                                 long long out_stride) {
    if (!ecs || !streams || nthreads < 1 || S < 0) return ECG_EINVAL;
    std::vector<int> rcs(nthreads, 0);
    std::vector<std::thread> th;
    th.reserve(nthreads);
    for (int t = 0; t < nthreads; t++) {
        const int c0 = (int)((long long)S * t / nthreads), c1 = (int)((long long)S * (t + 1) / nthreads);
        th.emplace_back([=, &rcs] {
            rcs[t] = ecg_replay_partial_repair(ecs[t], form, scope_stripes, base, sstride, bstride, B, c1 - c0,
                                               stripe_of + c0, pattern_of + c0, fail, n_surv, surv, n_help, help,
                                               n_main, main_, partials + 2LL * c0 * B, out, out_stride, streams[t]);
        });
    }
    for (auto& x : th) x.join();
    for (int rc : rcs)
        if (rc) return rc;
    return 0;
}

// Config 4's stripe merging as the proxies issue it (merge.cpp:1310-1402): per merge and merged-stripe row,
// the helper proxy's encode_partial_blocks_for_encoding over the old stripe it holds, through a handle of the
// stripe's own code with merged-stripe block ids (help_recal, handle_merge.cpp:380-381,453-454; PC maps them
// to row-code columns, pc.cpp:257-285), then the main proxy's own partial through an RS(x k1, m1) row-code
// handle with column indices (main_plan.ec_type = RS, merge.cpp:1327-1335; handle_merge.cpp:13-14,269-270),
// then perform_addition of the two partials into the new row parity (:319).  Merge s's blocks at
// base + s * sstride + b * bstride; row r's helper blocks help[r * n_help ..] with ids help_idx[..] and parity
// id help_parity[r], its main blocks main_[r * n_main ..] with columns main_idx[..] and parity column
// main_parity[r]; the partials of (merge s, row r) at partials + ((s * rows + r) * 2 + j) * B; the new parity
// at out + s * out_sstride + r * out_bstride.  Forms as ecg_replay_partial_repair (scopes of scope_merges
// merges).  Asynchronous on `stream`; returns 0 or the first negative ecg_* status.
int ecg_replay_merge(ecg_ec* main_ec, ecg_ec* help_ec, int form, int scope_merges, char* base, long long sstride,
                     long long bstride, int B, int S, int rows, int n_main, const int* main_, const int* main_idx,
                     const int* main_parity, int n_help, const int* help, const int* help_idx, const int* help_parity,
                     char* partials, char* out, long long out_sstride, long long out_bstride, void* stream) {
    if (!main_ec || !help_ec || form < 0 || form > 2 || B <= 0 || S < 0 || rows < 1 || n_main < 1 || n_help < 1 ||
        (form > 0 && scope_merges < 1))
        return ECG_EINVAL;
    int rc = ecg_ec_set_memory(main_ec, ECG_MEM_DEVICE, stream);
    if (!rc) rc = ecg_ec_set_memory(help_ec, ECG_MEM_DEVICE, stream);
    if (rc) return rc;
    std::vector<char*> hp(n_help), mp(n_main);
    auto merge = [&](int s) -> int {
        char* blk0 = base + (long long)s * sstride;
        for (int r = 0; r < rows; r++) {
            for (int j = 0; j < n_help; j++) hp[j] = blk0 + (long long)help[r * n_help + j] * bstride;
            for (int j = 0; j < n_main; j++) mp[j] = blk0 + (long long)main_[r * n_main + j] * bstride;
            char* pp[2] = {partials + ((long long)s * rows + r) * 2 * B,
                           partials + (((long long)s * rows + r) * 2 + 1) * B};
            int r1 = ecg_ec_encode_partial_blocks_for_encoding(help_ec, hp.data(), &pp[0], B, help_idx + r * n_help,
                                                               n_help, help_parity + r, 1);
            if (r1) return r1;
            r1 = ecg_ec_encode_partial_blocks_for_encoding(main_ec, mp.data(), &pp[1], B, main_idx + r * n_main,
                                                           n_main, main_parity + r, 1);
            if (r1) return r1;
            char* o = out + (long long)s * out_sstride + (long long)r * out_bstride;
            if ((r1 = ecg_ec_perform_addition(main_ec, pp, &o, B, 2, 1))) return r1;
        }
        return 0;
    };
    if (form == 0) {
        for (int s = 0; s < S; s++)
            if ((rc = merge(s))) return rc;
        return 0;
    }
    for (int c0 = 0; c0 < S; c0 += scope_merges) {
        const int c1 = c0 + scope_merges < S ? c0 + scope_merges : S;
        if ((rc = ecg_batch_begin())) return rc;
        if (form == 2 &&
            (rc = ecg_batch_scratch(partials + (long long)c0 * rows * 2 * B, (size_t)(c1 - c0) * rows * 2 * B))) {
            ecg_batch_end();
            return rc;
        }
        for (int s = c0; s < c1 && !rc; s++) rc = merge(s);
        const int re = ecg_batch_end();
        if (rc) return rc;
        if (re) return re;
    }
    return 0;
}

// Any per-stripe sequence of ErasureCode calls, for bench.py's `families` workload (every code class the
// reference builds, ec_factory metadata.cpp:48-77: encode, repair through generate_repair_plan's help blocks,
// degraded-read decode).  Stripe s (of S) runs the calls of pattern pattern_of[s]; pattern p's calls are
// prog[off[p] .. off[p + 1]), each call packed as
//   [kind, handle, n_in, in ids.., n_out, out ids.., n_a, a.., n_b, b.., n_c, c..]
// kind 0 encode(in = k data blocks, out = m coding blocks)                              erasure_code.h:86
//      1 encode_partial_blocks_for_decoding(in, out; a = local_survivor_idxs, b = survivor_idxs,
//        c = failure_idxs)                                                              handle_repair.cpp:249,566
//      2 perform_addition(in = partials, out; a = [block_num, parity_num])              handle_repair.cpp:375
//      3 decode(in = k data blocks, out = m coding blocks; a = erasures incl. the -1 (copied per call: the LRC
//        local path writes into it, lrc.cpp:35-38), b = [failed_num])                   proxy.cpp:666
//      4 encode_partial_blocks_for_encoding(in, out; a = data_idxs, b = parity_idxs)    handle_merge.cpp:453
// Block ids below nb are the stripe's blocks (base + s * sstride + id * bstride); ids nb .. nb + nscr - 1 are
// the stripe's scratch slots (scratch + (s * nscr + id - nb) * B), e.g. the partials a repair adds.  Calls run
// in batch scopes of scope_stripes stripes (0 = every call on its own), with the scratch slots of the scope
// declared ecg_batch_scratch when use_scratch (the partials of a repair then compose away).  Every handle is
// set to device memory on `stream`.  Returns 0 or the first negative status.
int ecg_replay_calls(ecg_ec** handles, int n_handles, int scope_stripes, int use_scratch, char* base, long long sstride,
                     long long bstride, int B, int S, const int* pattern_of, const int* prog, const int* off, int nb,
                     int nscr, char* scratch, void* stream) {
    if (!handles || n_handles < 1 || B <= 0 || S < 0 || nb < 1 || nscr < 0 || scope_stripes < 0 || !prog || !off)
        return ECG_EINVAL;
    for (int h = 0; h < n_handles; h++)
        if (int rc = ecg_ec_set_memory(handles[h], ECG_MEM_DEVICE, stream)) return rc;
    std::vector<char*> in, out;
    std::vector<int> er;
    auto blk = [&](int s, int id) -> char* {
        return id < nb ? base + (long long)s * sstride + (long long)id * bstride
                       : scratch + ((long long)s * nscr + (id - nb)) * B;
    };
    auto stripe = [&](int s) -> int {
        const int p = pattern_of ? pattern_of[s] : 0;
        for (int i = off[p]; i < off[p + 1];) {
            const int* c = prog + i;
            const int kind = c[0], h = c[1];
            if (h < 0 || h >= n_handles) return ECG_EINVAL;
            ecg_ec* ec = handles[h];
            const int n_in = c[2];
            const int* ids_in = c + 3;
            const int n_out = c[3 + n_in];
            const int* ids_out = c + 4 + n_in;
            const int* q = ids_out + n_out;
            const int n_a = q[0];
            const int* a = q + 1;
            const int n_b = a[n_a];
            const int* b = a + n_a + 1;
            const int n_c = b[n_b];
            const int* cc = b + n_b + 1;
            i += 4 + n_in + n_out + 3 + n_a + n_b + n_c;
            in.resize(n_in);
            out.resize(n_out);
            for (int j = 0; j < n_in; j++) in[j] = blk(s, ids_in[j]);
            for (int j = 0; j < n_out; j++) out[j] = blk(s, ids_out[j]);
            int rc;
            switch (kind) {
                case 0: rc = ecg_ec_encode(ec, in.data(), out.data(), B); break;
                case 1:
                    rc = ecg_ec_encode_partial_blocks_for_decoding(ec, in.data(), out.data(), B, a, n_a, b, n_b, cc, n_c);
                    break;
                case 2: rc = n_a == 2 ? ecg_ec_perform_addition(ec, in.data(), out.data(), B, a[0], a[1]) : ECG_EINVAL; break;
                case 3:
                    er.assign(a, a + n_a);
                    rc = n_b == 1 ? ecg_ec_decode(ec, in.data(), out.data(), B, er.data(), b[0]) : ECG_EINVAL;
                    break;
                case 4: rc = ecg_ec_encode_partial_blocks_for_encoding(ec, in.data(), out.data(), B, a, n_a, b, n_b); break;
                default: rc = ECG_EINVAL;
            }
            if (rc) return rc;
        }
        return 0;
    };
    int rc = 0;
    if (scope_stripes == 0) {
        for (int s = 0; s < S && !rc; s++) rc = stripe(s);
        return rc;
    }
    for (int c0 = 0; c0 < S; c0 += scope_stripes) {
        const int c1 = c0 + scope_stripes < S ? c0 + scope_stripes : S;
        if ((rc = ecg_batch_begin())) return rc;
        if (use_scratch && nscr > 0 &&
            (rc = ecg_batch_scratch(scratch + (long long)c0 * nscr * B, (size_t)(c1 - c0) * nscr * B))) {
            ecg_batch_end();
            return rc;
        }
        for (int s = c0; s < c1 && !rc; s++) rc = stripe(s);
        const int re = ecg_batch_end();
        if (rc) return rc;
        if (re) return re;
    }
    return 0;
}

// Config 1's per-stripe host calls (proxy.cpp:312-349: one jerasure_matrix_encode per stripe on the
// proxy's host buffers): data [S][k][B], coding [S][m][B] in host memory.  mode 0: one synchronous call
// per stripe; mode 1: the same calls inside batch scopes of `per_scope` stripes with host deferral on
// (ecg_batch_defer_host), the outputs written at each scope's end.
int ecg_replay_host_encode(int k, int m, const int* matrix, char* data, char* coding, int B, int S, int mode,
                           int per_scope) {
    if (k < 1 || m < 1 || B < 0 || S < 0 || mode < 0 || mode > 1 || (mode == 1 && per_scope < 1)) return ECG_EINVAL;
    std::vector<char*> dp(k), cp(m);
    auto one = [&](int s) {
        for (int j = 0; j < k; j++) dp[j] = data + ((long long)s * k + j) * B;
        for (int j = 0; j < m; j++) cp[j] = coding + ((long long)s * m + j) * B;
        return ecg_jerasure_matrix_encode(k, m, 8, (int*)matrix, dp.data(), cp.data(), B);
    };
    int rc = 0;
    if (mode == 0) {
        for (int s = 0; s < S && !rc; s++) rc = one(s);
        return rc;
    }
    for (int s0 = 0; s0 < S && !rc; s0 += per_scope) {
        if ((rc = ecg_batch_begin())) return rc;
        rc = ecg_batch_defer_host(1);
        for (int s = s0; s < S && s < s0 + per_scope && !rc; s++) rc = one(s);
        const int re = ecg_batch_end();
        if (!rc) rc = re;
    }
    return rc;
}

}  // extern "C"
