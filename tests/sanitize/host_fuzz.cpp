// Host-side fuzz driver for the sanitizer build (tools/sanitize_host.sh): exercises every CPU-only part of
// the C ABI -- matrix builders, Gauss-Jordan, decode planning (through the ErasureCode facade's matrix
// hooks), partitions, repair plans, index helpers -- over randomly drawn parameters, with the host
// translation units compiled under -fsanitize=address,undefined.  No GPU call is made.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ecg.h"
#include "engine.hpp"  // ecg::form_runs, ecg::PtrSet (pure host logic of the batch-scope flush)

static std::mt19937_64 rng(12345);
static int rnd(int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); }

static void matrices() {
    for (int t = 0; t < 300; t++) {
        const int k = rnd(1, 60), m = rnd(1, 12);
        int* v = ecg_reed_sol_vandermonde_coding_matrix(k, m, 8);
        int* c = ecg_cauchy_good_general_coding_matrix(k, m, 8);
        int* o = ecg_cauchy_original_coding_matrix(k, m, 8);
        if (o) ecg_cauchy_improve_coding_matrix(k, m, 8, o);
        if (v) {
            std::vector<int> r((size_t)k * m);
            for (auto& x : r) x = rnd(0, 255);
            ecg_free(ecg_jerasure_matrix_multiply(v, r.data(), m, k, k, m, 8));      // (m x k)(k x m)
            int* bad = ecg_jerasure_matrix_multiply(v, r.data(), m, k, m, k, 8);  // c1 = k vs r2 = m
            if (bad && k != m) abort();                                          // a mismatch is refused
            ecg_free(bad);
        }
        ecg_free(v);
        ecg_free(c);
        ecg_free(o);
        const int n = rnd(1, 24);
        std::vector<int> a((size_t)n * n), inv((size_t)n * n);
        for (auto& x : a) x = rnd(0, 3) ? rnd(0, 255) : 0;
        (void)ecg_jerasure_invert_matrix(a.data(), inv.data(), n, 8);
    }
    for (int e = 0; e < 256; e++) (void)ecg_cauchy_n_ones(e, 8);
    // edge arguments
    ecg_free(ecg_reed_sol_vandermonde_coding_matrix(0, 4, 8));
    ecg_free(ecg_reed_sol_vandermonde_coding_matrix(200, 57, 8));
    ecg_free(ecg_reed_sol_vandermonde_coding_matrix(4, 2, 16));
    ecg_free(ecg_jerasure_matrix_multiply(nullptr, nullptr, 1, 1, 1, 1, 8));
}

static ecg_coding_parameters params(int t) {
    ecg_coding_parameters cp{};
    switch (t) {
        case 0: cp.k = rnd(1, 30); cp.m = rnd(1, 6); break;
        case 1: cp.k = rnd(2, 10); cp.m = rnd(1, 4); cp.x = rnd(2, 4); cp.seri_num = rnd(0, cp.x - 1); break;
        case 2: case 5: cp.l = rnd(1, 4); cp.k = cp.l * rnd(2, 5); cp.g = rnd(t == 5 ? 2 : 1, 4); break;
        case 3: cp.l = rnd(2, 4); cp.k = (cp.l - 1) * rnd(2, 5); cp.g = rnd(1, 3); break;
        case 4: case 6: {
            cp.l = rnd(1, 4);
            cp.g = rnd(t == 6 ? 2 : 1, 4);
            const int kg = cp.l * rnd(std::max(2, (cp.g + 2 + cp.l - 1) / cp.l), 6);
            cp.k = kg - cp.g;
            break;
        }
        default:
            cp.k1 = rnd(2, 5); cp.m1 = rnd(1, 2); cp.k2 = rnd(2, 4); cp.m2 = rnd(1, 2);
            cp.x = rnd(2, 3); cp.seri_num = rnd(0, cp.x - 1);
    }
    return cp;
}

static void facade() {
    std::vector<int> buf(1 << 16);
    char info[256];
    for (int trial = 0; trial < 600; trial++) {
        const int t = rnd(0, 9);
        ecg_coding_parameters cp = params(t);
        cp.local_or_column = rnd(0, 1);
        ecg_ec* ec = ecg_ec_factory(t, &cp);
        if (!ec) continue;
        ecg_ec_init_coding_parameters(ec, &cp);
        ecg_coding_parameters back{};
        ecg_ec_get_coding_parameters(ec, &back);
        const int k = ecg_ec_k(ec), m = ecg_ec_m(ec), n = k + m;
        std::vector<int> M((size_t)k * m + 64);
        (void)ecg_ec_make_encoding_matrix(ec, M.data());
        (void)ecg_ec_self_information(ec, info, sizeof info);
        for (int rule = 0; rule < 4; rule++) {
            ecg_ec_set_placement_rule(ec, rule);
            ecg_ec_set_random_seed(ec, (unsigned long long)trial * 7 + rule);
            if (ecg_ec_generate_partition(ec) < 0) continue;
            const int len = ecg_ec_get_partition(ec, buf.data(), (int)buf.size());
            if (len > 0 && len <= (int)buf.size()) ecg_ec_set_partition(ec, buf.data(), len);
            (void)ecg_ec_grouping_information(ec, buf.data(), (int)buf.size());
            for (int f = 1; f <= std::min(4, m); f++) {
                std::vector<int> ids(n);
                for (int i = 0; i < n; i++) ids[i] = i;
                std::shuffle(ids.begin(), ids.end(), rng);
                ids.resize(f);
                int dec = -1;
                (void)ecg_ec_check_if_decodable(ec, ids.data(), f);
                (void)ecg_ec_generate_repair_plan(ec, ids.data(), f, buf.data(), (int)buf.size(), &dec);
            }
        }
        for (int b = -1; b <= n; b++) {
            int row = 0, col = 0, mn = 0;
            (void)ecg_ec_bid2gid(ec, b);
            (void)ecg_ec_idxingroup(ec, b);
            (void)ecg_ec_get_group_size(ec, b, &mn);
            (void)ecg_ec_bid2rowcol(ec, b, &row, &col);
            (void)ecg_ec_rowcol2bid(ec, row, col);
        }
        // partial coding matrices over random index subsets (the decode / encode planners)
        for (int r = 0; r < 6; r++) {
            std::vector<int> all(n);
            for (int i = 0; i < n; i++) all[i] = i;
            std::shuffle(all.begin(), all.end(), rng);
            const int nf = rnd(1, std::max(1, std::min(3, m)));
            std::vector<int> fail(all.begin(), all.begin() + nf);
            std::vector<int> surv(all.begin() + nf, all.begin() + std::min(n, nf + k));
            const int nl = rnd(1, (int)surv.size());
            std::vector<int> loc(surv.begin(), surv.begin() + nl);
            std::vector<int> out((size_t)nf * nl + 8);
            (void)ecg_ec_partial_decoding_matrix(ec, loc.data(), nl, surv.data(), (int)surv.size(), fail.data(), nf,
                                                 out.data(), (int)out.size());
            const int nd = rnd(1, k);
            std::vector<int> data(nd), par;
            for (int i = 0; i < nd; i++) data[i] = rnd(0, k - 1);
            for (int i = k; i < n; i++)
                if (rnd(0, 1)) par.push_back(i);
            if (par.empty()) par.push_back(n - 1);
            std::vector<int> out2(par.size() * (size_t)nd + 8);
            (void)ecg_ec_partial_encoding_matrix(ec, data.data(), nd, par.data(), (int)par.size(), out2.data(),
                                                 (int)out2.size());
        }
        ecg_ec_destroy(ec);
    }
}

// Decode planning (the symbolic replay of jerasure_matrix_decode and the facade's decode control flow)
// runs before any byte moves; without a GPU the execution step then fails cleanly with ECG_EHIP.
static void decode_plans() {
    const int B = 32;
    for (int t = 0; t < 400; t++) {
        const int k = rnd(1, 16), m = rnd(1, 6);
        std::vector<int> M((size_t)k * m);
        int* v = ecg_reed_sol_vandermonde_coding_matrix(k, m, 8);
        for (size_t i = 0; i < M.size(); i++) M[i] = (v && rnd(0, 2)) ? v[i] : rnd(0, 3) ? rnd(0, 255) : rnd(0, 1);
        ecg_free(v);
        std::vector<std::vector<char>> blocks(k + m, std::vector<char>(B, 1));
        std::vector<char*> p(k + m);
        for (int i = 0; i < k + m; i++) p[i] = blocks[i].data();
        std::vector<int> ids(k + m);
        for (int i = 0; i < k + m; i++) ids[i] = i;
        std::shuffle(ids.begin(), ids.end(), rng);
        const int f = rnd(1, std::min(k + m, m + 1));
        std::vector<int> er(ids.begin(), ids.begin() + f);
        er.push_back(-1);
        (void)ecg_jerasure_matrix_decode(k, m, 8, M.data(), rnd(0, 1), er.data(), p.data(), p.data() + k, B);
    }
    for (int trial = 0; trial < 300; trial++) {
        const int t = rnd(0, 9);
        ecg_coding_parameters cp = params(t);
        cp.local_or_column = rnd(0, 1);
        ecg_ec* ec = ecg_ec_factory(t, &cp);
        if (!ec) continue;
        ecg_ec_init_coding_parameters(ec, &cp);
        const int k = ecg_ec_k(ec), m = ecg_ec_m(ec), n = k + m;
        std::vector<std::vector<char>> blocks(n, std::vector<char>(B, 1));
        std::vector<char*> p(n);
        for (int i = 0; i < n; i++) p[i] = blocks[i].data();
        std::vector<int> ids(n);
        for (int i = 0; i < n; i++) ids[i] = i;
        std::shuffle(ids.begin(), ids.end(), rng);
        const int f = rnd(1, std::min(n, 4));
        std::vector<int> er(ids.begin(), ids.begin() + f);
        er.push_back(cp.local_or_column ? rnd(0, std::max(0, cp.l - 1)) : -1);  // LRC local: group id side channel
        er.push_back(-1);
        (void)ecg_ec_decode(ec, p.data(), p.data() + k, B, er.data(), f);
        ecg_ec_destroy(ec);
    }
}

// Run formation of the batch-scope flush (ecg::form_runs) against a quadratic restatement of its rule,
// over many runs per flush so PtrSet's clear / shrink / grow paths all execute under the sanitizers.
static void run_formation() {
    struct Call {
        int plan;
        std::vector<const void*> rd, wr;
    };
    long long runs_seen = 0;
    for (int trial = 0; trial < 400; trial++) {
        const int n = rnd(1, trial % 10 == 0 ? 6000 : 300);
        const int plans = rnd(1, 3);
        // pool: addresses shared between calls (hazards) or mostly private (long runs, big tables)
        const int pool = rnd(0, 2) ? n * 12 : rnd(2, 40);
        std::vector<Call> c(n);
        for (auto& x : c) {
            x.plan = rnd(0, plans - 1) * (rnd(0, 9) == 0 ? 1 : 0);
            const int nr = rnd(0, 5), nw = rnd(1, 3);
            for (int i = 0; i < nr; i++) x.rd.push_back((const void*)(uintptr_t)(0x1000 + 16 * rnd(0, pool)));
            for (int i = 0; i < nw; i++) x.wr.push_back((const void*)(uintptr_t)(0x1000 + 16 * rnd(0, pool)));
        }
        auto same = [&](size_t i, size_t j) { return c[i].plan == c[j].plan; };
        auto reads = [&](size_t i, auto&& f) { for (auto p : c[i].rd) f(p); };
        auto writes = [&](size_t i, auto&& f) { for (auto p : c[i].wr) f(p); };
        const std::vector<size_t> ends = ecg::form_runs((size_t)n, same, reads, writes);
        // quadratic reference: extend while the plan matches and no earlier call of the run conflicts
        size_t i = 0, r = 0;
        while (i < (size_t)n) {
            size_t j = i + 1;
            for (; j < (size_t)n && c[j].plan == c[i].plan; j++) {
                bool clash = false;
                for (size_t e = i; e < j && !clash; e++) {
                    for (auto p : c[j].rd) clash |= std::count(c[e].wr.begin(), c[e].wr.end(), p) > 0;
                    for (auto p : c[j].wr)
                        clash |= std::count(c[e].wr.begin(), c[e].wr.end(), p) + std::count(c[e].rd.begin(), c[e].rd.end(), p) > 0;
                }
                if (clash) break;
            }
            if (r >= ends.size() || ends[r] != j) {
                fprintf(stderr, "form_runs mismatch: trial %d run %zu\n", trial, r);
                abort();
            }
            i = j;
            r++;
        }
        if (r != ends.size()) abort();
        runs_seen += (long long)r;
    }
    // PtrSet alone: grow past 1024 slots, shrink on clear, duplicates, membership after regrowth
    ecg::PtrSet s;
    for (int round = 0; round < 6; round++) {
        const int cnt = round % 2 ? 20000 : 7;
        for (int i = 1; i <= cnt; i++) s.insert((const void*)(uintptr_t)(i * 48));
        for (int i = 1; i <= cnt; i++) s.insert((const void*)(uintptr_t)(i * 48));
        if (s.size() != (size_t)cnt) abort();
        for (int i = 1; i <= cnt; i++)
            if (!s.contains((const void*)(uintptr_t)(i * 48))) abort();
        if (s.contains((const void*)(uintptr_t)(cnt * 48 + 48))) abort();
        s.clear();
        if (s.size() != 0 || s.contains((const void*)(uintptr_t)48)) abort();
    }
    printf("run formation: %lld runs checked\n", runs_seen);
}

// Deferred-batch scope bookkeeping (record, hazard-split runs, strided-run detection) over fake device
// addresses.  Only where no GPU exists: the flush then stops at its first launch with ECG_EHIP (a
// program-table allocation), so only the first run is launched; the run boundaries of every flush are
// covered by run_formation() above.  With a GPU the fake addresses would be launched.
static void batch_scope() {
    if (ecg_device_count() > 0) return;
    ecg_coding_parameters cp{};
    cp.k = 6;
    cp.m = 3;
    ecg_ec* ec = ecg_ec_factory(ECG_RS, &cp);
    ecg_ec_set_memory(ec, ECG_MEM_DEVICE, nullptr);
    for (int trial = 0; trial < 40; trial++) {
        const int S = rnd(1, 3000), n = 9;
        const int pool = rnd(1, 4) == 1 ? S * n : S * n * 3;  // sometimes shared blocks: hazards split runs
        std::vector<char*> ptrs((size_t)S * n);
        for (int s = 0; s < S; s++)
            for (int b = 0; b < n; b++) {
                const size_t slot = rnd(0, 3) ? (size_t)s * n + b : (size_t)rnd(0, pool - 1);
                ptrs[(size_t)s * n + b] = (char*)(uintptr_t)(0x100000000ULL + slot * 4096);
            }
        if (ecg_batch_begin() != 0) abort();
        for (int s = 0; s < S; s++) ecg_ec_encode(ec, &ptrs[(size_t)s * n], &ptrs[(size_t)s * n + 6], 4096);
        const int rc = ecg_batch_end();
        if (rc != 0 && rc != ECG_EHIP) abort();
    }
    ecg_ec_destroy(ec);
}

int main() {
    matrices();
    facade();
    decode_plans();
    run_formation();
    batch_scope();
    printf("host fuzz done\n");
    return 0;
}
