// Host-side fuzz driver for the sanitizer build (tools/sanitize_host.sh): exercises every CPU-only part of
// the C ABI -- matrix builders, Gauss-Jordan, decode planning (through the ErasureCode facade's matrix
// hooks), partitions, repair plans, index helpers -- over randomly drawn parameters, with the host
// translation units compiled under -fsanitize=address,undefined.  No GPU call is made.
#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ecg.h"
#include "engine.hpp"  // ecg::schedule_groups, ecg::compose_scratch (pure host logic of the batch-scope flush)
#include "gf256.hpp"
#include "matrix.hpp"  // ecg::compose_chain

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

// Grouping of the batch-scope flush (ecg::schedule_groups) against a quadratic legality check: every call
// lands in exactly one group of its own key, dependent calls (write-after-read, read-after-write,
// write-after-write on one address) sit in strictly ordered groups, and the group count equals a
// quadratic restatement of the join rule.  Many groups per flush, so PtrGroups grows under the sanitizers.
static void grouping() {
    struct Call {
        int key;
        std::vector<const void*> rd, wr;
    };
    long long groups_seen = 0;
    for (int trial = 0; trial < 400; trial++) {
        const int n = rnd(1, trial % 10 == 0 ? 6000 : 300);
        const int keys = rnd(1, 16);
        // pool: addresses shared between calls (dependences) or mostly private (large groups, big tables)
        const int pool = rnd(0, 2) ? n * 12 : rnd(2, 40);
        std::vector<Call> c(n);
        for (auto& x : c) {
            x.key = rnd(0, keys - 1);
            const int nr = rnd(0, 5), nw = rnd(1, 3);
            for (int i = 0; i < nr; i++) x.rd.push_back((const void*)(uintptr_t)(0x1000 + 16 * rnd(0, pool)));
            for (int i = 0; i < nw; i++) x.wr.push_back((const void*)(uintptr_t)(0x1000 + 16 * rnd(0, pool)));
        }
        auto key = [&](size_t i) { return c[i].key; };
        auto reads = [&](size_t i, auto&& f) { for (auto p : c[i].rd) f(p); };
        auto writes = [&](size_t i, auto&& f) { for (auto p : c[i].wr) f(p); };
        const auto groups = ecg::schedule_groups((size_t)n, key, reads, writes);
        std::vector<int> g_of(n, -1);
        for (size_t g = 0; g < groups.size(); g++) {
            if (groups[g].empty()) abort();
            for (size_t i = 0; i < groups[g].size(); i++) {
                const size_t x = groups[g][i];
                if (g_of[x] != -1 || c[x].key != c[groups[g][0]].key) abort();
                if (i && groups[g][i - 1] >= x) abort();  // program order inside a group
                g_of[x] = (int)g;
            }
        }
        auto dep = [&](size_t a, size_t b) {  // b (later) depends on a
            for (auto p : c[b].rd) if (std::count(c[a].wr.begin(), c[a].wr.end(), p)) return true;
            for (auto p : c[b].wr)
                if (std::count(c[a].wr.begin(), c[a].wr.end(), p) || std::count(c[a].rd.begin(), c[a].rd.end(), p)) return true;
            return false;
        };
        // quadratic restatement of the join rule (the earliest group of the call's key after every group it
        // depends on, else a new group), and the legality of the result
        std::vector<int> ref(n);
        std::vector<std::vector<int>> mine(keys);
        int ng = 0;
        for (int b = 0; b < n; b++) {
            int lo = -1;
            for (int a = 0; a < b; a++) {
                if (g_of[a] == -1) abort();
                if (dep((size_t)a, (size_t)b)) {
                    if (g_of[a] >= g_of[b]) {
                        fprintf(stderr, "schedule_groups: dependence %d -> %d not ordered (trial %d)\n", a, b, trial);
                        abort();
                    }
                    lo = std::max(lo, ref[a]);
                }
            }
            ref[b] = -1;
            for (int g : mine[c[b].key])
                if (g > lo) {
                    ref[b] = g;
                    break;
                }
            if (ref[b] < 0) mine[c[b].key].push_back(ref[b] = ng++);
            if (ref[b] != g_of[b]) {
                fprintf(stderr, "schedule_groups: call %d in group %d, rule says %d (trial %d)\n", b, g_of[b], ref[b], trial);
                abort();
            }
        }
        if ((size_t)ng != groups.size()) abort();
        groups_seen += ng;
    }
    printf("grouping: %lld groups checked\n", groups_seen);
}

// Scratch composition (ecg::compose_scratch) + grouping against a sequential interpreter over real host
// bytes: random multi-op calls over a pool of 8-byte blocks, some of them scratch, some calls on a second
// "stream".  The composed calls, run in program order AND in the scheduler's group order, must leave every
// non-scratch block as the recorded calls run one by one do (and every block, scratch included, for a
// mid-scope flush, which writes leftover expressions out).  Engines and streams are never dereferenced.
static void scratch_composition() {
    constexpr int BS = 8;
    auto run_op = [&](const ecg::LinearOp& op, uint8_t* const* blocks) {  // read all inputs, then write
        std::vector<std::array<uint8_t, BS>> o(op.m_out());
        for (int p = 0; p < op.m_out(); p++) {
            o[p].fill(0);
            for (int j = 0; j < op.k_in(); j++)
                for (int x = 0; x < BS; x++)
                    o[p][x] ^= (uint8_t)ecg::gf::mul(op.coef[(size_t)p * op.k_in() + j], blocks[op.src_ids[j]][x]);
        }
        for (int p = 0; p < op.m_out(); p++) memcpy(blocks[op.dst_ids[p]], o[p].data(), BS);
    };
    ecg::Engine* eng = (ecg::Engine*)(uintptr_t)0x10;
    long long mats = 0, calls_in = 0, calls_out = 0;
    for (int trial = 0; trial < 3000; trial++) {
        const int P = rnd(2, 24), n = rnd(1, std::min(60, 2 + trial / 40));
        std::vector<uint8_t> mem0((size_t)P * BS);
        for (auto& b : mem0) b = (uint8_t)rnd(0, 255);
        ecg::ScratchRanges scr;
        std::vector<char> is_scr(P, 0);
        for (int b = 0; b < P; b++)
            if (rnd(0, 2) == 0) {
                is_scr[b] = 1;
                scr.add((uintptr_t)&mem0[(size_t)b * BS], (uintptr_t)&mem0[(size_t)b * BS] + BS);
            }
        std::vector<ecg::DeferredCall> q;
        for (int i = 0; i < n; i++) {
            const int nb = rnd(2, 6);
            ecg::DeferredCall c{eng, (hipStream_t)(uintptr_t)(rnd(0, 7) == 0 ? 2 : 1), BS, nullptr, {}};
            for (int b = 0; b < nb; b++) c.blocks.push_back(&mem0[(size_t)rnd(0, P - 1) * BS]);
            auto ops = std::make_shared<std::vector<ecg::LinearOp>>();
            const int nops = rnd(1, 2);
            for (int o = 0; o < nops; o++) {
                ecg::LinearOp op;
                const int k = rnd(1, nb - 1), m = rnd(1, std::min(3, nb - k));
                std::vector<int> ids(nb);
                for (int b = 0; b < nb; b++) ids[b] = b;
                std::shuffle(ids.begin(), ids.end(), rng);
                op.src_ids.assign(ids.begin(), ids.begin() + k);
                op.dst_ids.assign(ids.begin() + k, ids.begin() + k + m);
                if (rnd(0, 4) == 0) op.dst_ids[0] = op.src_ids[0];  // in place (galois_region_xor shape)
                for (int x = 0; x < k * m; x++) op.coef.push_back((uint8_t)(rnd(0, 3) == 0 ? 0 : rnd(0, 1) ? 1 : rnd(0, 255)));
                ops->push_back(op);
            }
            c.ops = ops;
            q.push_back(c);
        }
        const bool scope_end = rnd(0, 1);
        // one trial: false (and a dump if `verbose`) when a composed order differs from the sequential one
        auto verify = [&](const std::vector<ecg::DeferredCall>& q, bool verbose) {
            std::vector<uint8_t> ref = mem0;
            auto rebase = [&](uint8_t* p, std::vector<uint8_t>& m) { return m.data() + (p - mem0.data()); };
            for (auto& c : q) {
                std::vector<uint8_t*> bl;
                for (auto p : c.blocks) bl.push_back(rebase(p, ref));
                for (auto& op : *c.ops) run_op(op, bl.data());
            }
            long long nm = 0;
            std::vector<ecg::DeferredCall> q2 = ecg::compose_scratch(std::vector<ecg::DeferredCall>(q), scr, scope_end, &nm);
            if (!verbose) {
                mats += nm;
                calls_in += (long long)q.size();
                calls_out += (long long)q2.size();
            }
            auto dump = [&](const std::vector<ecg::DeferredCall>& v, const char* name) {
                fprintf(stderr, "%s:\n", name);
                for (auto& c : v) {
                    fprintf(stderr, " st%d", (int)(uintptr_t)c.st);
                    for (auto& op : *c.ops) {
                        fprintf(stderr, " [");
                        for (int p = 0; p < op.m_out(); p++) {
                            const long d = (long)((c.blocks[op.dst_ids[p]] - mem0.data()) / BS);
                            fprintf(stderr, " b%ld%s=", d, is_scr[d] ? "s" : "");
                            for (int j = 0; j < op.k_in(); j++)
                                fprintf(stderr, "%d*b%d+", op.coef[(size_t)p * op.k_in() + j],
                                        (int)((c.blocks[op.src_ids[j]] - mem0.data()) / BS));
                        }
                        fprintf(stderr, " ]");
                    }
                    fprintf(stderr, "\n");
                }
            };
            auto same = [&](std::vector<uint8_t>& got, const char* what) {
                for (int b = 0; b < P; b++) {
                    if (scope_end && is_scr[b]) continue;
                    if (memcmp(&got[(size_t)b * BS], &ref[(size_t)b * BS], BS)) {
                        if (verbose) {
                            fprintf(stderr, "scratch composition (%s, scope_end %d): block %d differs, trial %d\n", what,
                                    (int)scope_end, b, trial);
                            dump(q, "recorded");
                            dump(q2, "composed");
                        }
                        return false;
                    }
                }
                return true;
            };
            std::vector<uint8_t> seq = mem0;
            for (auto& c : q2) {
                std::vector<uint8_t*> bl;
                for (auto p : c.blocks) bl.push_back(rebase(p, seq));
                for (auto& op : *c.ops) run_op(op, bl.data());
            }
            if (!same(seq, "program order")) return false;
            // group order: key = plan content + stream
            std::vector<int> key(q2.size());
            std::vector<std::pair<const std::vector<ecg::LinearOp>*, hipStream_t>> seen;
            for (size_t i = 0; i < q2.size(); i++) {
                int id = -1;
                for (size_t s = 0; s < seen.size(); s++) {
                    const auto& a = *seen[s].first;
                    const auto& b = *q2[i].ops;
                    bool eq = a.size() == b.size() && seen[s].second == q2[i].st;
                    for (size_t o = 0; eq && o < a.size(); o++)
                        eq = a[o].src_ids == b[o].src_ids && a[o].dst_ids == b[o].dst_ids && a[o].coef == b[o].coef;
                    if (eq) id = (int)s;
                }
                if (id < 0) {
                    id = (int)seen.size();
                    seen.emplace_back(q2[i].ops.get(), q2[i].st);
                }
                key[i] = id;
            }
            auto reads = [&](size_t c, auto&& f) { for (auto& op : *q2[c].ops) for (int id : op.src_ids) f(q2[c].blocks[id]); };
            auto writes = [&](size_t c, auto&& f) { for (auto& op : *q2[c].ops) for (int id : op.dst_ids) f(q2[c].blocks[id]); };
            const auto groups = ecg::schedule_groups(q2.size(), [&](size_t c) { return key[c]; }, reads, writes);
            std::vector<uint8_t> grp = mem0;
            for (auto& G : groups)
                for (size_t o = 0; o < q2[G[0]].ops->size(); o++) {
                    // one launch: every call of the group reads before any call writes (independent calls)
                    std::vector<std::vector<uint8_t>> snap;
                    for (size_t c : G) {
                        std::vector<uint8_t> tmp = grp;
                        std::vector<uint8_t*> bl;
                        for (auto p : q2[c].blocks) bl.push_back(rebase(p, tmp));
                        run_op((*q2[c].ops)[o], bl.data());
                        snap.push_back(tmp);
                    }
                    for (size_t i = 0; i < G.size(); i++) {
                        const ecg::LinearOp& op = (*q2[G[i]].ops)[o];
                        for (int id : op.dst_ids) {
                            const size_t off = (size_t)(q2[G[i]].blocks[id] - mem0.data());
                            memcpy(&grp[off], &snap[i][off], BS);
                        }
                    }
                }
            return same(grp, "group order");
        };
        if (!verify(q, false)) {  // shrink to a minimal failing call list, then show it
            for (bool shrunk = true; shrunk;) {
                shrunk = false;
                for (size_t i = 0; i < q.size() && !shrunk; i++) {
                    std::vector<ecg::DeferredCall> r = q;
                    r.erase(r.begin() + (long)i);
                    if (!verify(r, false)) {
                        q = r;
                        shrunk = true;
                    }
                }
            }
            verify(q, true);
            abort();
        }
    }
    printf("scratch composition: %lld calls in, %lld out, %lld expressions materialised\n", calls_in, calls_out, mats);
}

// Deferred-batch scope bookkeeping (record, hazard-split runs, strided-run detection) over fake device
// addresses.  Only where no GPU exists: the flush then stops at its first launch with ECG_EHIP (a
// program-table allocation), so only the first group is launched; the grouping of every flush is
// covered by grouping() above.  With a GPU the fake addresses would be launched.
// Chain composition (ecg::compose_chain, the facade's product-code plans) against running the chain op by op:
// random chains over a small block-id space -- ops reading blocks earlier ops wrote, rewriting blocks, 0 / 1 /
// general coefficients, cancelling terms -- on random bytes.  Where compose_chain gives one op, that op over the
// original blocks must leave every block as the chain does; where it refuses, the chain must really need its
// order (a written block's original bytes feed a final value) or every final value is zero.
static void chains() {
    long long composed = 0, refused = 0;
    const int L = 37;
    for (int trial = 0; trial < 20000; trial++) {
        const int nb = rnd(2, 12), nops = rnd(1, 6);
        std::vector<ecg::LinearOp> ops(nops);
        for (auto& op : ops) {  // destinations, then sources from the other blocks: an op never reads what it writes
            std::vector<int> ids(nb);
            for (int i = 0; i < nb; i++) ids[i] = i;
            std::shuffle(ids.begin(), ids.end(), rng);
            const int m = rnd(1, std::min(4, nb - 1)), k = rnd(1, nb - m);
            op.dst_ids.assign(ids.begin(), ids.begin() + m);
            op.src_ids.assign(ids.begin() + m, ids.begin() + m + k);
            op.coef.resize(op.src_ids.size() * op.dst_ids.size());
            const int flavour = rnd(0, 2);
            for (auto& c : op.coef) c = (uint8_t)(flavour == 0 ? rnd(0, 1) : flavour == 1 ? rnd(0, 255) : (rnd(0, 3) ? 1 : rnd(2, 255)));
        }
        std::vector<std::vector<uint8_t>> seq(nb, std::vector<uint8_t>(L));
        for (auto& b : seq)
            for (auto& x : b) x = (uint8_t)rnd(0, 255);
        const std::vector<std::vector<uint8_t>> orig = seq;
        auto apply = [&](const ecg::LinearOp& op, const std::vector<std::vector<uint8_t>>& in,
                         std::vector<std::vector<uint8_t>>& out) {
            std::vector<std::vector<uint8_t>> rows(op.m_out(), std::vector<uint8_t>(L, 0));
            for (int p = 0; p < op.m_out(); p++)
                for (int j = 0; j < op.k_in(); j++)
                    for (int x = 0; x < L; x++)
                        rows[p][x] ^= (uint8_t)ecg::gf::mul(op.coef[(size_t)p * op.k_in() + j], in[op.src_ids[j]][x]);
            for (int p = 0; p < op.m_out(); p++) out[op.dst_ids[p]] = rows[p];
        };
        for (const auto& op : ops) apply(op, seq, seq);
        ecg::LinearOp one;
        if (!ecg::compose_chain(ops, one)) {
            refused++;
            continue;
        }
        composed++;
        for (int s : one.src_ids)
            if (std::find(one.dst_ids.begin(), one.dst_ids.end(), s) != one.dst_ids.end()) {
                fprintf(stderr, "compose_chain: composed op reads a block it writes (trial %d)\n", trial);
                abort();
            }
        std::vector<std::vector<uint8_t>> got = orig;
        apply(one, orig, got);
        if (got != seq) {
            fprintf(stderr, "compose_chain: composed op differs from the chain (trial %d)\n", trial);
            abort();
        }
    }
    printf("chains: %lld composed and checked, %lld left as chains\n", composed, refused);
}

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
    if (const char* e = getenv("ECG_FUZZ_SEED")) rng.seed(strtoull(e, nullptr, 10));
    matrices();
    facade();
    decode_plans();
    grouping();
    scratch_composition();
    chains();
    batch_scope();
    printf("host fuzz done\n");
    return 0;
}
