// Loopback harness: coordinator-lite + proxy-lite over the C ABI.  See loopback.hpp for scope.
#include "loopback.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <thread>

#include "wire.hpp"

namespace ecg_loopback {

namespace {

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::string key_of(unsigned block_id) { return std::to_string(block_id); }

bool is_lrc(int t) { return t >= ECG_AZURE_LRC && t <= ECG_UNIFORM_CAUCHY_LRC; }
bool is_pc(int t) { return t == ECG_PC || t == ECG_HIERACHICAL_PC || t == ECG_HV_PC; }

// One ErasureCode object per call, as the proxies build them (ec_factory + init_coding_parameters,
// handle_repair.cpp:13-14), on host buffers: every byte operation runs on the GPU engine.
struct Ec {
    ecg_ec* h = nullptr;
    Ec(int type, ecg_coding_parameters cp) {
        h = ecg_ec_factory(type, &cp);
        if (h) {
            ecg_ec_init_coding_parameters(h, &cp);
            ecg_ec_set_memory(h, ECG_MEM_HOST, nullptr);
        }
    }
    ~Ec() {
        if (h) ecg_ec_destroy(h);
    }
    Ec(const Ec&) = delete;
    Ec& operator=(const Ec&) = delete;
};

struct BlockLoc {
    int idx;            // index in the coding space of the call (block index, or row / column for PCs)
    unsigned block_id;  // datanode key
    unsigned node;
};

struct RepairCall {  // MainRepairPlan / HelpRepairPlan (metadata.h:136-200)
    int ec_type = ECG_RS;
    ecg_coding_parameters cp{};
    int cluster_id = 0;
    size_t block_size = 0;
    bool partial_decoding = true;
    std::vector<int> live, failed;
    std::vector<unsigned> failed_ids;
    std::vector<BlockLoc> inner;                    // blocks inside this proxy's cluster
    std::vector<std::vector<BlockLoc>> help;        // main only: blocks of every helper cluster
    std::vector<unsigned> new_nodes;                // main only
};

struct RecalCall {  // MainRecalPlan / HelpRecalPlan (metadata.h:202-230)
    int ec_type = ECG_RS;
    ecg_coding_parameters cp{};
    int cluster_id = 0;
    size_t block_size = 0;
    bool partial_decoding = true;
    std::vector<int> parity_idx;
    std::vector<unsigned> new_parity_ids, new_nodes;  // main only
    std::vector<BlockLoc> inner;
    std::vector<std::vector<BlockLoc>> help;          // main only
};

using Block = std::vector<char>;

std::vector<char*> ptrs(std::vector<Block>& v) {
    std::vector<char*> p(v.size());
    for (size_t i = 0; i < v.size(); i++) p[i] = v[i].data();
    return p;
}

}  // namespace

struct Loopback::Impl {
    Loopback& L;
    EcSchema schema;
    Topology topo;
    BlockStore& store;
    std::mt19937_64 rng;
    unsigned cur_stripe_id = 0, cur_block_id = 0;
    std::vector<std::vector<unsigned>> merge_groups;

    Impl(Loopback& l, const EcSchema& s, const Topology& t, BlockStore& st, uint64_t seed)
        : L(l), schema(s), topo(t), store(st), rng(seed) {}

    int random_index(size_t n) { return n ? (int)(rng() % n) : 0; }

    // ECG_EUNDECODABLE from a decode = the matrix the library picked is singular: for the non-MDS LRCs
    // the reference's check_if_decodable accepts patterns that are not (e.g. Azure(12,2,2) losing data
    // blocks 0,1,2: global row 0 and local row 0 coincide on them), and its decode prints "[Decode]
    // Failed!" (lrc.cpp:52-55).  Counted apart from real errors.
    bool ok(int rc) {
        if (rc == ECG_EUNDECODABLE) L.stats.decode_undecodable++;
        else if (rc < 0) L.stats.ecg_errors++;
        return rc >= 0;
    }

    bool read(const BlockLoc& b, size_t B, Block& out) {
        out.assign(B, 0);
        return store.access_data(topo.node_port(b.node), key_of(b.block_id), out.data(), B);
    }

    // ------------------------------------------------------------ proxy-lite: repair

    // Proxy::help_repair (handle_repair.cpp:472-650): partial decoding over the cluster's blocks, sent
    // to the main proxy as [cid][1][f][f x B][seconds].
    bool help_repair(const RepairCall& p, Channel& main) {
        const int f = (int)p.failed.size();
        Ec ec(p.ec_type, p.cp);
        const bool partial = ec.h && p.partial_decoding && (int)p.live.size() <= ecg_ec_k(ec.h);
        if (ec.h && !(partial && (int)p.inner.size() > f)) return true;  // the main proxy reads them directly
        Bytes msg;
        const bool good = ec.h && help_repair_partial(p, ec.h, msg);
        if (!good) {
            msg.clear();
            put_int(msg, p.cluster_id);
            put_int(msg, -1);
        }
        main.send(std::move(msg));
        return good;
    }

    bool help_repair_partial(const RepairCall& p, ecg_ec* ec, Bytes& msg) {
        const int f = (int)p.failed.size();
        std::vector<Block> data(p.inner.size()), coding(f, Block(p.block_size));
        std::vector<int> idx;
        for (size_t i = 0; i < p.inner.size(); i++) {
            if (!read(p.inner[i], p.block_size, data[i])) return false;
            idx.push_back(p.inner[i].idx);
        }
        auto dp = ptrs(data), cpp = ptrs(coding);
        const double t0 = now_s();
        if (!ok(ecg_ec_encode_partial_blocks_for_decoding(ec, dp.data(), cpp.data(), (int)p.block_size, idx.data(),
                                                          (int)idx.size(), p.live.data(), (int)p.live.size(),
                                                          p.failed.data(), f)))
            return false;
        const double t = now_s() - t0;
        put_int(msg, p.cluster_id);
        put_int(msg, 1);
        put_int(msg, f);
        for (auto& c : coding) put_bytes(msg, c.data(), c.size());
        put_double(msg, t);
        return true;
    }

    // Proxy::main_repair (handle_repair.cpp:5-470).  Returns the rebuilt blocks in failed order.
    std::string last_kind;  // how the latest main_repair ran

    bool main_repair(const RepairCall& p, Channel& chan, std::vector<Block>& out) {
        const int f = (int)p.failed.size();
        const size_t B = p.block_size;
        Ec ec(p.ec_type, p.cp);
        if (!ec.h) return false;
        const int ek = ecg_ec_k(ec.h), em = ecg_ec_m(ec.h);
        const bool partial = p.partial_decoding && (int)p.live.size() <= ek;
        std::vector<Block> orig;
        std::vector<int> orig_idx;
        auto take = [&](const BlockLoc& b) {
            Block v;
            if (!read(b, B, v)) return false;
            orig.push_back(std::move(v));
            orig_idx.push_back(b.idx);
            return true;
        };
        for (auto& b : p.inner)
            if (!take(b)) return false;
        int expect = 0;
        for (auto& cluster : p.help) {
            if (partial && (int)cluster.size() > f) {
                expect++;
            } else {
                for (auto& b : cluster)  // IF_DIRECT_FROM_NODE (metadata.h:14)
                    if (!take(b)) return false;
            }
        }
        std::vector<Block> partials;
        bool helpers_ok = true;
        for (int i = 0; i < expect; i++) {  // drain every helper's frame before deciding
            Bytes msg = chan.accept();
            if (msg.size() < 2 * sizeof(int)) {
                helpers_ok = false;
                continue;
            }
            Reader r(msg);
            r.get_int();  // helper cluster id
            if (r.get_int() != 1 || r.get_int() != f) {
                helpers_ok = false;
                continue;
            }
            for (int j = 0; j < f; j++) {
                Block v(B);
                r.get_bytes(v.data(), B);
                partials.push_back(std::move(v));
            }
            r.get_double();
            if (!r.done()) helpers_ok = false;
            L.stats.helper_messages++;
            L.stats.helper_bytes += (long)msg.size();
        }
        if (!helpers_ok) return false;
        out.assign(f, Block(B, 0));
        last_kind = std::string(partial ? "partial-" : "direct-") + (p.cp.local_or_column ? "local" : "global");
        if (partial) {
            // The main cluster's own partial over its blocks, then perform_addition with the helpers'
            // partials (handle_repair.cpp:371-376), done as ONE call: the own partial never round-trips.
            auto op = ptrs(out);
            if (partials.empty()) {
                if (orig.empty()) return false;
                auto dp = ptrs(orig);
                if (!ok(ecg_ec_encode_partial_blocks_for_decoding(ec.h, dp.data(), op.data(), (int)B, orig_idx.data(),
                                                                  (int)orig_idx.size(), p.live.data(),
                                                                  (int)p.live.size(), p.failed.data(), f)))
                    return false;
            } else if (orig.empty() && (int)partials.size() == f) {
                out = partials;
            } else {
                auto dp = ptrs(orig), pp = ptrs(partials);
                if (!ok(ecg_ec_encode_partial_blocks_for_decoding_with_addition(
                        ec.h, dp.data(), pp.data(), (int)partials.size(), op.data(), (int)B, orig_idx.data(),
                        (int)orig_idx.size(), p.live.data(), (int)p.live.size(), p.failed.data(), f)))
                    return false;
            }
            L.stats.plans_partial++;
            return true;
        }
        L.stats.plans_direct++;
        if (is_lrc(p.ec_type) && p.cp.local_or_column) {  // local decode in group space (:296-345, :372-378)
            if (f != 1) return false;
            ecg_coding_parameters cp{};
            ecg_ec_get_coding_parameters(ec.h, &cp);
            const int kg = cp.k + cp.g;
            int group_id = -1;
            for (int i : p.live)
                if (i >= kg) {
                    group_id = i - kg;
                    break;
                }
            if (group_id < 0)
                for (int i : p.failed)
                    if (i >= kg) group_id = i - kg;
            if (group_id < 0) group_id = ecg_ec_bid2gid(ec.h, p.failed[0]);
            int min_idx = 0;
            const int gs = ecg_ec_get_group_size(ec.h, group_id, &min_idx);
            if (gs < 0) return false;
            auto slot = [&](int idx) {
                if (idx >= kg) return gs;
                if (idx >= cp.k && p.ec_type == ECG_OPTIMAL_CAUCHY_LRC) return gs - cp.g + (idx - cp.k);
                return ecg_ec_idxingroup(ec.h, idx);
            };
            std::vector<Block> data(std::max<size_t>(gs, p.live.size()), Block(B, 0)), coding(1, Block(B, 0));
            for (size_t i = 0; i < orig.size(); i++) {
                const int s = slot(orig_idx[i]);
                (s >= gs ? coding[s - gs] : data[s]) = orig[i];
            }
            const int fs = slot(p.failed[0]);
            int erasures[2] = {fs, group_id};
            auto dp = ptrs(data), cpp = ptrs(coding);
            if (!ok(ecg_ec_decode(ec.h, dp.data(), cpp.data(), (int)B, erasures, 1))) return false;
            out[0] = fs >= gs ? coding[fs - gs] : data[fs];
            return true;
        }
        // global decode over the blocks that were read: every other block is an erasure (the reference
        // lists only the failed blocks and leaves unread buffers as null pointers, :275-282, 347-356)
        std::vector<Block> data(ek, Block(B, 0)), coding(em, Block(B, 0));
        std::vector<char> have(ek + em, 0);
        for (size_t i = 0; i < orig.size(); i++) {
            const int idx = orig_idx[i];
            (idx < ek ? data[idx] : coding[idx - ek]) = orig[i];
            have[idx] = 1;
        }
        std::vector<int> erasures;
        for (int i = 0; i < ek + em; i++)
            if (!have[i]) erasures.push_back(i);
        const int n_er = (int)erasures.size();
        erasures.push_back(-1);
        auto dp = ptrs(data), cpp = ptrs(coding);
        if (!ok(ecg_ec_decode(ec.h, dp.data(), cpp.data(), (int)B, erasures.data(), n_er))) return false;
        for (int i = 0; i < f; i++) out[i] = p.failed[i] < ek ? data[p.failed[i]] : coding[p.failed[i] - ek];
        return true;
    }

    // ------------------------------------------------------------ coordinator-lite: repair

    // auxs.cpp:139-159: partitions = the clusters the stripe's blocks actually sit in (the reference
    // iterates an unordered_map; here clusters in order of their first block)
    void find_out_stripe_partitions(Stripe& s) {
        std::vector<int> order;
        std::map<int, std::vector<int>> by_cluster;
        for (int i = 0; i < s.k + s.m; i++) {
            const int c = topo.cluster_of(s.blocks2nodes[i]);
            if (!by_cluster.count(c)) order.push_back(c);
            by_cluster[c].push_back(i);
        }
        std::vector<int> flat{(int)order.size()};
        for (int c : order) {
            flat.push_back((int)by_cluster[c].size());
            flat.insert(flat.end(), by_cluster[c].begin(), by_cluster[c].end());
        }
        ecg_ec_set_partition(s.ec, flat.data(), (int)flat.size());
    }

    struct Plan {
        bool local_or_column;
        std::vector<int> failures;
        std::vector<std::vector<int>> help;
    };

    bool plans_of(Stripe& s, const std::vector<int>& failures, std::vector<Plan>& plans) {
        int dec = 0;
        int need = ecg_ec_generate_repair_plan(s.ec, failures.data(), (int)failures.size(), nullptr, 0, &dec);
        if (need < 0 || !dec) return false;
        std::vector<int> buf(need);
        ecg_ec_generate_repair_plan(s.ec, failures.data(), (int)failures.size(), buf.data(), need, &dec);
        int at = 1;
        for (int i = 0; i < buf[0]; i++) {
            Plan p;
            p.local_or_column = buf[at++] != 0;
            const int nf = buf[at++];
            p.failures.assign(buf.begin() + at, buf.begin() + at + nf);
            at += nf;
            const int nh = buf[at++];
            for (int h = 0; h < nh; h++) {
                const int sz = buf[at++];
                p.help.emplace_back(buf.begin() + at, buf.begin() + at + sz);
                at += sz;
            }
            plans.push_back(p);
        }
        return true;
    }

    // Proxy::decode_and_get_object's degraded read (proxy.cpp:517-666): partitions from the placement,
    // generate_repair_plan over the unreachable data blocks, fetch the plan's help blocks, then ONE
    // ec->decode with local_or_column = false (:564) and the unreachable blocks as erasures.
    // Two reference defects are fixed, not copied:
    //   * the reference fetches only the plan's help blocks but decodes GLOBALLY, so for a local plan
    //     (LRC single loss) the global decode reads coding buffers it never fetched (zeros); here the
    //     decode's own read set is fetched too: the first k surviving blocks (jerasure_matrix_decode),
    //     or every surviving block for the product codes' iterative decode;
    //   * proxy.cpp:673-677 never puts the rebuilt blocks into the returned value (a degraded GET there
    //     is short); here they are.
    bool degraded_read(Stripe& s, const std::vector<int>& obj_blocks, const std::vector<int>& missing,
                       std::vector<char>& value) {
        const size_t B = schema.block_size;
        const int n = s.k + s.m;
        std::vector<int> failures;
        for (int j : missing) failures.push_back(obj_blocks[j]);
        find_out_stripe_partitions(s);
        std::vector<Plan> plans;
        if (!plans_of(s, failures, plans)) return false;
        std::vector<Block> data(s.k, Block(B, 0)), coding(s.m, Block(B, 0));
        std::vector<char> have(n, 0), lost(n, 0), want(n, 0);
        for (int f : failures) lost[f] = 1;
        for (size_t j = 0; j < obj_blocks.size(); j++) {  // blocks the GET already read
            const int b = obj_blocks[j];
            if (lost[b]) continue;
            memcpy((b < s.k ? data[b] : coding[b - s.k]).data(), value.data() + j * B, B);
            have[b] = 1;
        }
        for (auto& p : plans)
            for (auto& h : p.help)
                for (int b : h) want[b] = 1;
        if (is_pc(schema.ec_type)) {
            for (int b = 0; b < n; b++) want[b] |= !lost[b];
        } else {
            for (int b = 0, got = 0; b < n && got < s.k; b++)
                if (!lost[b]) {
                    want[b] = 1;
                    got++;
                }
        }
        for (int b = 0; b < n; b++) {
            if (!want[b] || have[b] || lost[b]) continue;
            if (!read(BlockLoc{b, s.block_ids[b], s.blocks2nodes[b]}, B, b < s.k ? data[b] : coding[b - s.k]))
                return false;
            have[b] = 1;
        }
        ecg_coding_parameters saved{};
        ecg_ec_get_coding_parameters(s.ec, &saved);
        ecg_coding_parameters cp = saved;
        cp.local_or_column = 0;  // proxy.cpp:564
        ecg_ec_init_coding_parameters(s.ec, &cp);
        std::vector<int> erasures = failures;
        erasures.push_back(-1);
        auto dp = ptrs(data), cpp = ptrs(coding);
        const int rc = ecg_ec_decode(s.ec, dp.data(), cpp.data(), (int)B, erasures.data(), (int)failures.size());
        ecg_ec_init_coding_parameters(s.ec, &saved);
        if (!ok(rc)) return false;
        for (int j : missing) memcpy(value.data() + j * B, data[obj_blocks[j]].data(), B);
        return true;
    }

    // repair.cpp:190-470 concrete_repair_plans / concrete_repair_plans_pc
    bool concretise(Stripe& s, const Plan& plan, RepairCall& main, std::vector<RepairCall>& helps) {
        const int main_cid = topo.cluster_of(s.blocks2nodes[plan.failures[0]]);
        std::map<int, std::vector<unsigned>> free_nodes;
        for (int f : plan.failures) {
            const unsigned nid = s.blocks2nodes[f];
            const int c = topo.cluster_of(nid);
            if (!free_nodes.count(c))
                for (int j = 0; j < topo.nodes_per_cluster; j++)
                    free_nodes[c].push_back((unsigned)(c * topo.nodes_per_cluster + j));
            auto& fn = free_nodes[c];
            fn.erase(std::remove(fn.begin(), fn.end(), nid), fn.end());
        }
        const bool pc = is_pc(schema.ec_type);
        int k1 = 0, m1 = 0, k2 = 0, m2 = 0;
        ecg_coding_parameters scp{};
        ecg_ec_get_coding_parameters(s.ec, &scp);
        auto space_idx = [&](int bid) {  // PCs address a column (row index) or a row (column index)
            if (!pc) return bid;
            int r = -1, c = -1;
            ecg_ec_bid2rowcol(s.ec, bid, &r, &c);
            return plan.local_or_column ? r : c;
        };
        if (pc) {
            k1 = scp.k1, m1 = scp.m1, k2 = scp.k2, m2 = scp.m2;
            main.cp = ecg_coding_parameters{};
            main.cp.k = plan.local_or_column ? k2 : k1;
            main.cp.m = plan.local_or_column ? m2 : m1;
            main.ec_type = ECG_RS;
            if (schema.ec_type == ECG_HIERACHICAL_PC)  // HPC objects are vertical (pc.h:66): ERS columns
                main.ec_type = plan.local_or_column ? ECG_ERS : ECG_RS;  // repair.cpp:393-409
        } else {
            main.cp = scp;
            main.ec_type = schema.ec_type;
        }
        main.cp.x = schema.x;
        main.cp.seri_num = (int)(s.stripe_id % schema.x);
        main.cp.local_or_column = plan.local_or_column;
        main.cluster_id = main_cid;
        main.block_size = schema.block_size;
        main.partial_decoding = schema.partial_decoding;
        for (auto& hb : plan.help) {
            if (hb.empty()) continue;
            for (int b : hb) main.live.push_back(space_idx(b));
        }
        if (!pc && (int)main.live.size() > s.k) main.partial_decoding = false;  // repair.cpp:245-247
        for (int f : plan.failures) {
            main.failed.push_back(space_idx(f));
            main.failed_ids.push_back(s.block_ids[f]);
        }
        for (auto& hb : plan.help) {
            if (hb.empty()) continue;
            const int cid = topo.cluster_of(s.blocks2nodes[hb[0]]);
            std::vector<BlockLoc> locs;
            for (int b : hb) locs.push_back({space_idx(b), s.block_ids[b], s.blocks2nodes[b]});
            if (cid == main_cid) {
                for (auto& l : locs) {
                    main.inner.push_back(l);
                    auto it = free_nodes.find(cid);
                    if (it != free_nodes.end())
                        it->second.erase(std::remove(it->second.begin(), it->second.end(), l.node), it->second.end());
                }
            } else {
                RepairCall h;
                h.ec_type = main.ec_type;
                h.cp = main.cp;
                h.cluster_id = cid;
                h.block_size = main.block_size;
                h.partial_decoding = main.partial_decoding;
                h.failed = main.failed;
                h.live = main.live;
                h.inner = locs;
                main.help.push_back(locs);
                helps.push_back(h);
            }
        }
        for (int f : plan.failures) {
            auto& fn = free_nodes[topo.cluster_of(s.blocks2nodes[f])];
            if (fn.empty()) return false;
            const int at = random_index(fn.size());
            main.new_nodes.push_back(fn[at]);
            fn.erase(fn.begin() + at);
        }
        return true;
    }

    std::vector<std::string> kinds;  // plan kinds of the current repair

    bool run_plan(Stripe& s, const Plan& plan) {
        RepairCall main;
        std::vector<RepairCall> helps;
        if (!concretise(s, plan, main, helps)) return false;
        Channel chan;
        std::vector<std::thread> threads;
        std::vector<char> help_ok(helps.size(), 1);
        for (size_t i = 0; i < helps.size(); i++)
            threads.emplace_back([&, i] { help_ok[i] = help_repair(helps[i], chan); });
        std::vector<Block> rebuilt;
        last_kind.clear();
        const bool main_ok = main_repair(main, chan, rebuilt);
        if (!last_kind.empty()) kinds.push_back(last_kind);
        for (auto& t : threads) t.join();
        if (!main_ok || std::find(help_ok.begin(), help_ok.end(), 0) != help_ok.end()) return false;
        for (size_t i = 0; i < plan.failures.size(); i++) {  // send_to_datanode, then metadata follows
            const int bid = plan.failures[i];
            if (!store.store_data(topo.node_port(main.new_nodes[i]), key_of(s.block_ids[bid]), rebuilt[i].data(),
                                  rebuilt[i].size()))
                return false;
            s.blocks2nodes[bid] = main.new_nodes[i];
            L.stats.blocks_rebuilt++;
        }
        L.stats.repair_plans++;
        return true;
    }

    // ------------------------------------------------------------ proxy-lite: merge (recalculation)

    bool help_recal(const RecalCall& p, Channel& main) {  // handle_merge.cpp:362-538
        const int np = (int)p.parity_idx.size();
        if (!(p.partial_decoding && (int)p.inner.size() > np)) return true;
        Bytes msg;
        Ec ec(p.ec_type, p.cp);
        const bool good = ec.h && help_recal_partial(p, ec.h, msg);
        if (!good) {
            msg.clear();
            put_int(msg, p.cluster_id);
            put_int(msg, -1);
        }
        main.send(std::move(msg));
        return good;
    }

    bool help_recal_partial(const RecalCall& p, ecg_ec* ec, Bytes& msg) {
        const int np = (int)p.parity_idx.size();
        std::vector<Block> data(p.inner.size()), coding(np, Block(p.block_size));
        std::vector<int> idx;
        for (size_t i = 0; i < p.inner.size(); i++) {
            if (!read(p.inner[i], p.block_size, data[i])) return false;
            idx.push_back(p.inner[i].idx);
        }
        auto dp = ptrs(data), cpp = ptrs(coding);
        const double t0 = now_s();
        if (!ok(ecg_ec_encode_partial_blocks_for_encoding(ec, dp.data(), cpp.data(), (int)p.block_size, idx.data(),
                                                          (int)idx.size(), p.parity_idx.data(), np)))
            return false;
        put_int(msg, p.cluster_id);
        put_int(msg, 1);
        put_int(msg, np);
        for (auto& c : coding) put_bytes(msg, c.data(), c.size());
        put_double(msg, now_s() - t0);
        return true;
    }

    bool main_recal(const RecalCall& p, Channel& chan, std::vector<Block>& out) {  // handle_merge.cpp:5-360
        const int np = (int)p.parity_idx.size();
        const size_t B = p.block_size;
        Ec ec(p.ec_type, p.cp);
        if (!ec.h) return false;
        if (p.ec_type == ECG_HIERACHICAL_PC) {  // :100-157: new parity = XOR of the old ones (ERS rows)
            std::vector<Block> old(p.inner.size());
            for (size_t i = 0; i < p.inner.size(); i++)
                if (!read(p.inner[i], B, old[i])) return false;
            out.assign(np, Block(B, 0));
            auto dp = ptrs(old), op = ptrs(out);
            return ok(ecg_ec_perform_addition(ec.h, dp.data(), op.data(), (int)B, (int)old.size(), np));
        }
        std::vector<Block> orig;
        std::vector<int> orig_idx;
        auto take = [&](const BlockLoc& b) {
            Block v;
            if (!read(b, B, v)) return false;
            orig.push_back(std::move(v));
            orig_idx.push_back(b.idx);
            return true;
        };
        for (auto& b : p.inner)
            if (!take(b)) return false;
        int expect = 0;
        for (auto& cluster : p.help) {
            if (p.partial_decoding && (int)cluster.size() > np) {
                expect++;
            } else {
                for (auto& b : cluster)
                    if (!take(b)) return false;
            }
        }
        std::vector<Block> partials;
        bool helpers_ok = true;
        for (int i = 0; i < expect; i++) {
            Bytes msg = chan.accept();
            if (msg.size() < 2 * sizeof(int)) {
                helpers_ok = false;
                continue;
            }
            Reader r(msg);
            r.get_int();
            if (r.get_int() != 1 || r.get_int() != np) {
                helpers_ok = false;
                continue;
            }
            for (int j = 0; j < np; j++) {
                Block v(B);
                r.get_bytes(v.data(), B);
                partials.push_back(std::move(v));
            }
            r.get_double();
            if (!r.done()) helpers_ok = false;
            L.stats.helper_messages++;
            L.stats.helper_bytes += (long)msg.size();
        }
        if (!helpers_ok) return false;
        out.assign(np, Block(B, 0));
        auto op = ptrs(out);
        if (p.partial_decoding && !partials.empty()) {
            // own partial encoding + perform_addition (handle_merge.cpp:159,319) in one call
            auto dp = ptrs(orig), pp = ptrs(partials);
            return ok(ecg_ec_encode_partial_blocks_for_encoding_with_addition(
                ec.h, dp.data(), pp.data(), (int)partials.size(), op.data(), (int)B, orig_idx.data(),
                (int)orig_idx.size(), p.parity_idx.data(), np));
        }
        auto dp = ptrs(orig);
        return ok(ecg_ec_encode_partial_blocks_for_encoding(ec.h, dp.data(), op.data(), (int)B, orig_idx.data(),
                                                            (int)orig_idx.size(), p.parity_idx.data(), np));
    }

    // main_recal + help_recal of one parity-recalculation plan: helpers on their own threads, the main
    // proxy here (merge.cpp:405-425 / 1395-1415).
    bool run_recal(const RecalCall& main, const std::vector<RecalCall>& helps, std::vector<Block>& parities) {
        Channel chan;
        std::vector<std::thread> threads;
        std::vector<char> help_ok(helps.size(), 1);
        for (size_t i = 0; i < helps.size(); i++)
            threads.emplace_back([&, i] { help_ok[i] = help_recal(helps[i], chan); });
        bool good = main_recal(main, chan, parities);
        for (auto& t : threads) t.join();
        return good && std::find(help_ok.begin(), help_ok.end(), 0) == help_ok.end();
    }

    // group the (new index, block id, node) inputs of one recalculation by cluster, in order of first
    // appearance; the parity cluster's blocks are the main proxy's own, the others become helpers
    void split_recal(RecalCall& main, const std::vector<BlockLoc>& inputs, std::vector<RecalCall>& helps) {
        std::vector<std::pair<int, std::vector<BlockLoc>>> clusters;
        for (auto& b : inputs) {
            const int c = topo.cluster_of(b.node);
            auto it = std::find_if(clusters.begin(), clusters.end(), [&](auto& e) { return e.first == c; });
            if (it == clusters.end()) {
                clusters.push_back({c, {}});
                it = clusters.end() - 1;
            }
            it->second.push_back(b);
        }
        for (auto& c : clusters) {
            if (c.first == main.cluster_id) {
                main.inner.insert(main.inner.end(), c.second.begin(), c.second.end());
            } else {
                RecalCall h;
                h.ec_type = main.ec_type;
                h.cp = main.cp;
                h.cluster_id = c.first;
                h.block_size = main.block_size;
                h.partial_decoding = main.partial_decoding;
                h.parity_idx = main.parity_idx;
                h.inner = c.second;
                main.help.push_back(c.second);
                helps.push_back(h);
            }
        }
    }
};

// ================================================================ Loopback

Loopback::Loopback(const EcSchema& schema, const Topology& topo, BlockStore& store, uint64_t seed)
    : impl_(std::make_unique<Impl>(*this, schema, topo, store, seed)) {}

Loopback::~Loopback() {
    for (auto& kv : stripes_)
        if (kv.second.ec) ecg_ec_destroy(kv.second.ec);
}

std::vector<unsigned> Loopback::list_stripes() const {
    std::vector<unsigned> ids;
    for (auto& kv : stripes_) ids.push_back(kv.first);
    return ids;
}

bool Loopback::set(const std::string& key, const std::vector<char>& value) {
    Impl& I = *impl_;
    const double t0 = now_s();
    Stripe s;
    s.stripe_id = I.cur_stripe_id++;
    ecg_coding_parameters cp = I.schema.cp;
    cp.x = I.schema.x;
    cp.seri_num = (int)(s.stripe_id % I.schema.x);
    s.ec = ecg_ec_factory(I.schema.ec_type, &cp);
    if (!s.ec) return false;
    ecg_ec_init_coding_parameters(s.ec, &cp);
    ecg_ec_set_memory(s.ec, ECG_MEM_HOST, nullptr);
    s.k = ecg_ec_k(s.ec);
    s.m = ecg_ec_m(s.ec);
    const size_t B = I.schema.block_size;
    if (value.size() != (size_t)s.k * B) {
        ecg_ec_destroy(s.ec);
        return false;
    }
    for (int i = 0; i < s.k + s.m; i++) s.block_ids.push_back(I.cur_block_id++);
    // placement.cpp:5-140 (multistripe RAND): every partition in its own randomly chosen cluster,
    // every block on its own randomly chosen node of that cluster
    ecg_ec_set_placement_rule(s.ec, I.schema.placement_rule);
    ecg_ec_set_random_seed(s.ec, I.rng());
    if (ecg_ec_generate_partition(s.ec) != ECG_OK) return false;
    int need = ecg_ec_get_partition(s.ec, nullptr, 0);
    std::vector<int> flat(need);
    ecg_ec_get_partition(s.ec, flat.data(), need);
    s.blocks2nodes.assign(s.k + s.m, 0);
    std::vector<int> free_clusters(I.topo.clusters);
    for (int c = 0; c < I.topo.clusters; c++) free_clusters[c] = c;
    int at = 1;
    for (int p = 0; p < flat[0]; p++) {
        const int sz = flat[at++];
        if (free_clusters.empty()) return false;
        const int ci = I.random_index(free_clusters.size());
        const int c = free_clusters[ci];
        free_clusters.erase(free_clusters.begin() + ci);
        std::vector<unsigned> free_nodes;
        for (int j = 0; j < I.topo.nodes_per_cluster; j++) free_nodes.push_back((unsigned)(c * I.topo.nodes_per_cluster + j));
        for (int j = 0; j < sz; j++) {
            if (free_nodes.empty()) return false;
            const int ni = I.random_index(free_nodes.size());
            s.blocks2nodes[flat[at + j]] = free_nodes[ni];
            free_nodes.erase(free_nodes.begin() + ni);
        }
        at += sz;
    }
    // Proxy::encode_and_store_object (proxy.cpp:274-427)
    std::vector<Block> coding(s.m, Block(B));
    std::vector<char*> dp(s.k), cpp = ptrs(coding);
    for (int j = 0; j < s.k; j++) dp[j] = const_cast<char*>(value.data()) + j * B;
    if (!I.ok(ecg_ec_encode(s.ec, dp.data(), cpp.data(), (int)B))) return false;
    for (int j = 0; j < s.k + s.m; j++) {
        const char* src = j < s.k ? dp[j] : coding[j - s.k].data();
        if (!I.store.store_data(I.topo.node_port(s.blocks2nodes[j]), key_of(s.block_ids[j]), src, B)) return false;
    }
    s.objects.push_back(key);
    std::vector<int> data_blocks(s.k);
    for (int j = 0; j < s.k; j++) data_blocks[j] = j;
    objects_[key] = {s.stripe_id, data_blocks};
    if (I.merge_groups.empty() || (int)I.merge_groups.back().size() == I.schema.x) I.merge_groups.push_back({});
    I.merge_groups.back().push_back(s.stripe_id);
    stripes_[s.stripe_id] = s;
    stats.sets++;
    stats.set_s += now_s() - t0;
    return true;
}

bool Loopback::get(const std::string& key, std::vector<char>& value) {
    Impl& I = *impl_;
    const double t0 = now_s();
    auto it = objects_.find(key);
    if (it == objects_.end()) return false;
    const Stripe& s = stripes_.at(it->second.first);
    const std::vector<int>& blocks = it->second.second;
    const size_t B = I.schema.block_size;
    value.assign(blocks.size() * B, 0);
    std::vector<int> missing;  // positions in the value whose data block is unreachable
    for (size_t j = 0; j < blocks.size(); j++) {
        const int b = blocks[j];
        if (!I.store.access_data(I.topo.node_port(s.blocks2nodes[b]), key_of(s.block_ids[b]), value.data() + j * B, B))
            missing.push_back((int)j);
    }
    if (!missing.empty()) {
        if (!I.degraded_read(stripes_.at(it->second.first), blocks, missing, value)) return false;
        stats.degraded_gets++;
    }
    stats.gets++;
    stats.get_s += now_s() - t0;
    return true;
}

bool Loopback::get_with_unreachable(const std::string& key, int data_pos, std::vector<char>& value) {
    Impl& I = *impl_;
    auto it = objects_.find(key);
    if (it == objects_.end() || data_pos < 0 || data_pos >= (int)it->second.second.size()) return false;
    const Stripe& s = stripes_.at(it->second.first);
    const int b = it->second.second[data_pos];
    const size_t B = I.schema.block_size;
    const int port = I.topo.node_port(s.blocks2nodes[b]);
    Block keep(B);
    if (!I.store.access_data(port, key_of(s.block_ids[b]), keep.data(), B)) return false;
    I.store.remove_data(port, key_of(s.block_ids[b]));  // the datanode is unreachable
    const bool got = get(key, value);
    I.store.store_data(port, key_of(s.block_ids[b]), keep.data(), B);
    return got;
}

bool Loopback::repair(unsigned stripe_id, const std::vector<int>& failures) {
    Impl& I = *impl_;
    const double t0 = now_s();
    Stripe& s = stripes_.at(stripe_id);
    const size_t B = I.schema.block_size;
    if (ecg_ec_check_if_decodable(s.ec, failures.data(), (int)failures.size()) != 1) {
        stats.repairs_skipped_undecodable++;
        return false;
    }
    // the failure: the blocks are gone from their datanodes (kept aside to verify the rebuilt copies)
    std::vector<Block> lost(failures.size(), Block(B));
    std::vector<unsigned> lost_nodes;
    for (size_t i = 0; i < failures.size(); i++) {
        const int b = failures[i];
        lost_nodes.push_back(s.blocks2nodes[b]);
        const int port = I.topo.node_port(s.blocks2nodes[b]);
        if (!I.store.access_data(port, key_of(s.block_ids[b]), lost[i].data(), B)) return false;
        I.store.remove_data(port, key_of(s.block_ids[b]));
    }
    bool good = true;
    ecg_ec_set_placement_rule(s.ec, I.schema.placement_rule);  // repair.cpp:19-22
    ecg_ec_generate_partition(s.ec);
    I.find_out_stripe_partitions(s);
    std::vector<Impl::Plan> plans;
    I.kinds.clear();
    good = I.plans_of(s, failures, plans);
    for (auto& p : plans) {  // plans run in order; each is concretised after the previous one landed
        if (!good) break;
        good = I.run_plan(s, p);
        if (good) I.find_out_stripe_partitions(s);
    }
    bool recorded = false;
    for (size_t i = 0; i < failures.size(); i++) {
        const int b = failures[i];
        Block now(B);
        const bool found =
            I.store.access_data(I.topo.node_port(s.blocks2nodes[b]), key_of(s.block_ids[b]), now.data(), B);
        if (!good || !found || now != lost[i]) {
            if (good) {
                stats.rebuilt_mismatch++;
                if (!recorded) mismatches.push_back({stripe_id, failures, I.kinds});
                recorded = true;
            }
            // restore so the remaining sequence runs on intact data (drop a copy an earlier plan wrote)
            if (found && s.blocks2nodes[b] != lost_nodes[i])
                I.store.remove_data(I.topo.node_port(s.blocks2nodes[b]), key_of(s.block_ids[b]));
            s.blocks2nodes[b] = lost_nodes[i];
            I.store.store_data(I.topo.node_port(lost_nodes[i]), key_of(s.block_ids[b]), lost[i].data(), B);
        }
    }
    if (!good) stats.repairs_failed++;
    stats.repairs++;
    stats.repair_s += now_s() - t0;
    return good;
}

bool Loopback::merge(int step_size) {  // Coordinator::do_stripe_merge (merge.cpp:5-17)
    if (impl_->schema.ec_type == ECG_RS) return rs_merge(step_size);
    if (impl_->schema.ec_type == ECG_PC || impl_->schema.ec_type == ECG_HV_PC) return pc_merge(step_size);
    if (impl_->schema.ec_type == ECG_HIERACHICAL_PC) return hpc_merge(step_size);
    if (impl_->schema.ec_type == ECG_AZURE_LRC) return lrc_merge(step_size);
    return false;  // do_stripe_merge has no path for the other LRCs (merge.cpp:7-16)
}

bool Loopback::rs_merge(int step_size) {  // merge.cpp:19-450
    Impl& I = *impl_;
    const double t0 = now_s();
    const size_t B = I.schema.block_size;
    std::vector<std::vector<unsigned>> new_groups;
    bool all_ok = true;
    for (auto& group : I.merge_groups) {
        if ((int)group.size() % step_size != 0) continue;
        for (size_t mi = 0; mi < group.size(); mi += step_size) {
            Stripe big;
            big.stripe_id = I.cur_stripe_id++;
            std::vector<unsigned> parity_nodes, old_parity_ids, old_parity_nodes;
            std::vector<BlockLoc> inputs;  // data blocks under their merged-stripe index seri * k + i
            int k0 = 0, m0 = 0;
            for (int seri = 0; seri < step_size; seri++) {
                const Stripe& t = stripes_.at(group[mi + seri]);
                k0 = t.k;
                m0 = t.m;
                for (int i = 0; i < t.k + t.m; i++) {
                    const unsigned node = t.blocks2nodes[i];
                    if (i < t.k) {
                        big.blocks2nodes.push_back(node);
                        big.block_ids.push_back(t.block_ids[i]);
                        inputs.push_back({seri * t.k + i, t.block_ids[i], node});
                    } else {
                        parity_nodes.push_back(node);
                        old_parity_ids.push_back(t.block_ids[i]);
                        old_parity_nodes.push_back(node);
                    }
                }
            }
            ecg_coding_parameters cp = I.schema.cp;
            cp.k = k0 * step_size;  // Coordinator::new_ec_for_merge (auxs.cpp:102-120)
            cp.x = step_size;
            big.k = cp.k;
            big.m = m0;
            RecalCall main;
            main.ec_type = ECG_RS;
            main.cp = cp;
            main.block_size = B;
            main.partial_decoding = I.schema.partial_decoding;
            for (int i = 0; i < m0; i++) {  // new parities on the first stripe's parity nodes
                big.blocks2nodes.push_back(parity_nodes[i]);
                big.block_ids.push_back(I.cur_block_id++);
                main.cluster_id = I.topo.cluster_of(parity_nodes[i]);
                main.parity_idx.push_back(big.k + i);
                main.new_parity_ids.push_back(big.block_ids.back());
                main.new_nodes.push_back(parity_nodes[i]);
            }
            std::vector<RecalCall> helps;
            I.split_recal(main, inputs, helps);
            std::vector<Block> parities;
            if (!I.run_recal(main, helps, parities)) {
                all_ok = false;
                continue;
            }
            // old parities are deleted (DeletePlan), the new ones written in their place
            for (size_t i = 0; i < old_parity_ids.size(); i++)
                I.store.remove_data(I.topo.node_port(old_parity_nodes[i]), key_of(old_parity_ids[i]));
            for (int i = 0; i < m0; i++)
                I.store.store_data(I.topo.node_port(main.new_nodes[i]), key_of(main.new_parity_ids[i]),
                                   parities[i].data(), B);
            big.ec = ecg_ec_factory(ECG_RS, &cp);
            ecg_ec_init_coding_parameters(big.ec, &cp);
            ecg_ec_set_memory(big.ec, ECG_MEM_HOST, nullptr);
            for (int seri = 0; seri < step_size; seri++) {
                Stripe& t = stripes_.at(group[mi + seri]);
                for (auto& key : t.objects) {
                    big.objects.push_back(key);
                    std::vector<int> blocks(t.k);
                    for (int j = 0; j < t.k; j++) blocks[j] = seri * t.k + j;
                    objects_[key] = {big.stripe_id, blocks};
                }
                ecg_ec_destroy(t.ec);
                stripes_.erase(group[mi + seri]);
            }
            if (new_groups.empty() || (int)new_groups.back().size() == I.schema.x) new_groups.push_back({});
            new_groups.back().push_back(big.stripe_id);
            stripes_[big.stripe_id] = big;
            stats.merges++;
            stats.merged_parities += m0;
        }
    }
    I.merge_groups = new_groups;
    stats.merge_s += now_s() - t0;
    return all_ok;
}

// merge.cpp:877-1505 (PC, HVPC), multistripe rule HORIZONTAL
bool Loopback::pc_merge(int step_size) {
    Impl& I = *impl_;
    const double t0 = now_s();
    const size_t B = I.schema.block_size;
    const bool hv = I.schema.ec_type == ECG_HV_PC;
    std::vector<std::vector<unsigned>> new_groups;
    bool all_ok = true;
    for (auto& group : I.merge_groups) {
        if ((int)group.size() % step_size != 0) continue;
        for (size_t mi = 0; mi < group.size(); mi += step_size) {
            ecg_coding_parameters oc{};
            ecg_ec_get_coding_parameters(stripes_.at(group[mi]).ec, &oc);
            const int k1 = oc.k1, m1 = oc.m1, k2 = oc.k2, m2 = oc.m2, K1 = step_size * k1;
            ecg_coding_parameters nc = oc;  // Coordinator::new_ec_for_merge: k1 *= x (auxs.cpp:113-117)
            nc.k1 = K1;
            nc.x = step_size;
            Stripe big;
            big.stripe_id = I.cur_stripe_id++;
            big.ec = ecg_ec_factory(I.schema.ec_type, &nc);
            if (!big.ec) return false;
            ecg_ec_init_coding_parameters(big.ec, &nc);
            ecg_ec_set_memory(big.ec, ECG_MEM_HOST, nullptr);
            big.k = ecg_ec_k(big.ec);
            big.m = ecg_ec_m(big.ec);
            big.block_ids.assign(big.k + big.m, 0);
            big.blocks2nodes.assign(big.k + big.m, 0);
            const int rows = k2 + m2;
            std::vector<std::vector<BlockLoc>> row_inputs(rows);
            std::vector<std::vector<unsigned>> parity_nodes(rows, std::vector<unsigned>(m1, 0));
            std::vector<std::pair<unsigned, unsigned>> old_parities;  // (node, block id)
            for (int seri = 0; seri < step_size; seri++) {
                const Stripe& t = stripes_.at(group[mi + seri]);
                for (int i = 0; i < t.k + t.m; i++) {
                    int row = -1, col = -1;
                    ecg_ec_bid2rowcol(t.ec, i, &row, &col);
                    if (col < k1) {  // data and column-parity blocks keep their place in the wider grid
                        const int nb = ecg_ec_rowcol2bid(big.ec, row, seri * k1 + col);
                        big.block_ids[nb] = t.block_ids[i];
                        big.blocks2nodes[nb] = t.blocks2nodes[i];
                        row_inputs[row].push_back({seri * k1 + col, t.block_ids[i], t.blocks2nodes[i]});
                    } else {  // row parities and global parities are recomputed in place of the old ones
                        parity_nodes[row][col - k1] = t.blocks2nodes[i];
                        old_parities.push_back({t.blocks2nodes[i], t.block_ids[i]});
                    }
                }
            }
            bool ok = true;
            for (int row = 0; row < rows && ok; row++) {
                if (hv && row >= k2) continue;  // HVPC has no global parities (merge.cpp:1312-1321)
                RecalCall main;
                main.ec_type = ECG_RS;  // the row code RS(x * k1, m1)
                main.cp.k = K1;
                main.cp.m = m1;
                main.cp.x = step_size;
                main.block_size = B;
                main.partial_decoding = I.schema.partial_decoding;
                for (int ii = 0; ii < m1; ii++) {
                    const int nb = ecg_ec_rowcol2bid(big.ec, row, K1 + ii);
                    big.block_ids[nb] = I.cur_block_id++;
                    big.blocks2nodes[nb] = parity_nodes[row][ii];
                    main.parity_idx.push_back(K1 + ii);
                    main.new_parity_ids.push_back(big.block_ids[nb]);
                    main.new_nodes.push_back(parity_nodes[row][ii]);
                    main.cluster_id = I.topo.cluster_of(parity_nodes[row][ii]);
                }
                std::vector<RecalCall> helps;
                I.split_recal(main, row_inputs[row], helps);
                std::vector<Block> parities;
                ok = I.run_recal(main, helps, parities);
                for (int ii = 0; ok && ii < m1; ii++)
                    ok = I.store.store_data(I.topo.node_port(main.new_nodes[ii]), key_of(main.new_parity_ids[ii]),
                                            parities[ii].data(), B);
            }
            if (!ok) {
                all_ok = false;
                ecg_ec_destroy(big.ec);
                continue;
            }
            for (auto& op : old_parities) I.store.remove_data(I.topo.node_port(op.first), key_of(op.second));
            for (int seri = 0; seri < step_size; seri++) {
                Stripe& t = stripes_.at(group[mi + seri]);
                for (auto& key : t.objects) {  // an object's data: its old grid, columns shifted by seri * k1
                    big.objects.push_back(key);
                    std::vector<int> blocks;
                    for (int b : objects_.at(key).second) {
                        int row = -1, col = -1;
                        ecg_ec_bid2rowcol(t.ec, b, &row, &col);
                        blocks.push_back(ecg_ec_rowcol2bid(big.ec, row, seri * k1 + col));
                    }
                    objects_[key] = {big.stripe_id, blocks};
                }
                ecg_ec_destroy(t.ec);
                stripes_.erase(group[mi + seri]);
            }
            if (new_groups.empty() || (int)new_groups.back().size() == I.schema.x) new_groups.push_back({});
            new_groups.back().push_back(big.stripe_id);
            stripes_[big.stripe_id] = big;
            stats.merges++;
            stats.merged_parities += hv ? (long)k2 * m1 : (long)rows * m1;
        }
    }
    I.merge_groups = new_groups;
    stats.merge_s += now_s() - t0;
    return all_ok;
}

bool Loopback::lrc_merge(int step_size) {  // azu_lrc_merge, merge.cpp:451-877
    Impl& I = *impl_;
    const double t0 = now_s();
    const size_t B = I.schema.block_size;
    std::vector<std::vector<unsigned>> new_groups;
    bool all_ok = true;
    for (auto& group : I.merge_groups) {
        if ((int)group.size() % step_size != 0) continue;
        for (size_t mi = 0; mi < group.size(); mi += step_size) {
            ecg_coding_parameters oc{};
            ecg_ec_get_coding_parameters(stripes_.at(group[mi]).ec, &oc);
            const int k = oc.k, l = oc.l, g = oc.g;
            ecg_coding_parameters nc = oc;  // new_ec_for_merge: k *= x, l *= x (auxs.cpp:109-111)
            nc.k = step_size * k;
            nc.l = step_size * l;
            nc.m = nc.l + g;
            nc.x = step_size;
            nc.local_or_column = 0;
            Stripe big;
            big.stripe_id = I.cur_stripe_id++;
            big.ec = ecg_ec_factory(I.schema.ec_type, &nc);
            if (!big.ec) return false;
            ecg_ec_init_coding_parameters(big.ec, &nc);
            ecg_ec_set_memory(big.ec, ECG_MEM_HOST, nullptr);
            big.k = ecg_ec_k(big.ec);
            big.m = ecg_ec_m(big.ec);
            big.block_ids.assign(big.k + big.m, 0);
            big.blocks2nodes.assign(big.k + big.m, 0);
            std::vector<BlockLoc> inputs;
            std::vector<unsigned> parity_nodes;
            std::vector<std::pair<unsigned, unsigned>> old_globals;
            for (int seri = 0; seri < step_size; seri++) {
                const Stripe& t = stripes_.at(group[mi + seri]);
                for (int i = 0; i < t.k + t.m; i++) {
                    if (i < k || i >= k + g) {  // data and local parities keep their blocks
                        const int ni = i < k ? seri * k + i : big.k + g + seri * l + (i - k - g);
                        big.block_ids[ni] = t.block_ids[i];
                        big.blocks2nodes[ni] = t.blocks2nodes[i];
                        if (i < k) inputs.push_back({ni, t.block_ids[i], t.blocks2nodes[i]});
                    } else {
                        parity_nodes.push_back(t.blocks2nodes[i]);
                        old_globals.push_back({t.blocks2nodes[i], t.block_ids[i]});
                    }
                }
            }
            RecalCall main;
            main.ec_type = I.schema.ec_type;
            main.cp = nc;
            main.block_size = B;
            main.partial_decoding = I.schema.partial_decoding;
            for (int j = 0; j < g; j++) {  // the globals land on the first stripe's global nodes
                big.block_ids[big.k + j] = I.cur_block_id++;
                big.blocks2nodes[big.k + j] = parity_nodes[j];
                main.cluster_id = I.topo.cluster_of(parity_nodes[j]);
                main.parity_idx.push_back(big.k + j);
                main.new_parity_ids.push_back(big.block_ids[big.k + j]);
                main.new_nodes.push_back(parity_nodes[j]);
            }
            std::vector<RecalCall> helps;
            I.split_recal(main, inputs, helps);
            std::vector<Block> parities;
            bool ok = I.run_recal(main, helps, parities);
            for (int j = 0; ok && j < g; j++)
                ok = I.store.store_data(I.topo.node_port(main.new_nodes[j]), key_of(main.new_parity_ids[j]),
                                        parities[j].data(), B);
            if (!ok) {
                all_ok = false;
                ecg_ec_destroy(big.ec);
                continue;
            }
            for (auto& og : old_globals) I.store.remove_data(I.topo.node_port(og.first), key_of(og.second));
            for (int seri = 0; seri < step_size; seri++) {
                Stripe& t = stripes_.at(group[mi + seri]);
                for (auto& key : t.objects) {
                    big.objects.push_back(key);
                    std::vector<int> blocks;
                    for (int b : objects_.at(key).second) blocks.push_back(seri * k + b);
                    objects_[key] = {big.stripe_id, blocks};
                }
                ecg_ec_destroy(t.ec);
                stripes_.erase(group[mi + seri]);
            }
            if (new_groups.empty() || (int)new_groups.back().size() == I.schema.x) new_groups.push_back({});
            new_groups.back().push_back(big.stripe_id);
            stripes_[big.stripe_id] = big;
            stats.merges++;
            stats.merged_parities += g;
        }
    }
    I.merge_groups = new_groups;
    stats.merge_s += now_s() - t0;
    return all_ok;
}

// hpc_merge (merge.cpp:1505-1905), multistripe rule VERTICAL: HPC columns are ERS(k2, m2, x, seri)
// slices of one Vandermonde(x * k2, m2), so a merged column parity is the XOR of the x old ones, read
// by the parity's proxy (handle_merge.cpp:100-157); rows (data and row parities) keep their blocks.
bool Loopback::hpc_merge(int step_size) {
    Impl& I = *impl_;
    const double t0 = now_s();
    const size_t B = I.schema.block_size;
    std::vector<std::vector<unsigned>> new_groups;
    bool all_ok = true;
    for (auto& group : I.merge_groups) {
        if ((int)group.size() % step_size != 0) continue;
        for (size_t mi = 0; mi < group.size(); mi += step_size) {
            ecg_coding_parameters oc{};
            ecg_ec_get_coding_parameters(stripes_.at(group[mi]).ec, &oc);
            const int k1 = oc.k1, m1 = oc.m1, k2 = oc.k2, m2 = oc.m2, K2 = step_size * k2;
            ecg_coding_parameters nc = oc;  // new_ec_for_merge, VERTICAL: k2 *= x (auxs.cpp:113-115)
            nc.k2 = K2;
            nc.x = step_size;
            Stripe big;
            big.stripe_id = I.cur_stripe_id++;
            big.ec = ecg_ec_factory(ECG_HIERACHICAL_PC, &nc);
            if (!big.ec) return false;
            ecg_ec_init_coding_parameters(big.ec, &nc);
            ecg_ec_set_memory(big.ec, ECG_MEM_HOST, nullptr);
            big.k = ecg_ec_k(big.ec);
            big.m = ecg_ec_m(big.ec);
            big.block_ids.assign(big.k + big.m, 0);
            big.blocks2nodes.assign(big.k + big.m, 0);
            const int cols = k1 + m1;
            std::vector<std::vector<BlockLoc>> old_col_parities(cols);
            std::vector<std::vector<unsigned>> parity_nodes(cols, std::vector<unsigned>(m2, 0));
            std::vector<std::pair<unsigned, unsigned>> old_parities;
            for (int seri = 0; seri < step_size; seri++) {
                const Stripe& t = stripes_.at(group[mi + seri]);
                for (int i = 0; i < t.k + t.m; i++) {
                    int row = -1, col = -1;
                    ecg_ec_bid2rowcol(t.ec, i, &row, &col);
                    if (row < k2) {  // data and row parities: rows stack (oldbid2newbid_for_merge, pc.cpp:361-376)
                        const int nb = ecg_ec_rowcol2bid(big.ec, seri * k2 + row, col);
                        big.block_ids[nb] = t.block_ids[i];
                        big.blocks2nodes[nb] = t.blocks2nodes[i];
                    } else {
                        parity_nodes[col][row - k2] = t.blocks2nodes[i];
                        old_parities.push_back({t.blocks2nodes[i], t.block_ids[i]});
                        old_col_parities[col].push_back({seri * m2 + row - k2, t.block_ids[i], t.blocks2nodes[i]});
                    }
                }
            }
            bool ok = true;
            for (int col = 0; col < cols && ok; col++) {
                RecalCall main;
                main.ec_type = ECG_HIERACHICAL_PC;
                main.cp = nc;
                main.block_size = B;
                main.partial_decoding = I.schema.partial_decoding;
                main.inner = old_col_parities[col];
                for (int ii = 0; ii < m2; ii++) {
                    const int nb = ecg_ec_rowcol2bid(big.ec, K2 + ii, col);
                    big.block_ids[nb] = I.cur_block_id++;
                    big.blocks2nodes[nb] = parity_nodes[col][ii];
                    main.parity_idx.push_back(K2 + ii);
                    main.new_parity_ids.push_back(big.block_ids[nb]);
                    main.new_nodes.push_back(parity_nodes[col][ii]);
                    main.cluster_id = I.topo.cluster_of(parity_nodes[col][ii]);
                }
                std::vector<Block> parities;
                ok = I.run_recal(main, {}, parities);
                for (int ii = 0; ok && ii < m2; ii++)
                    ok = I.store.store_data(I.topo.node_port(main.new_nodes[ii]), key_of(main.new_parity_ids[ii]),
                                            parities[ii].data(), B);
            }
            if (!ok) {
                all_ok = false;
                ecg_ec_destroy(big.ec);
                continue;
            }
            for (auto& op : old_parities) I.store.remove_data(I.topo.node_port(op.first), key_of(op.second));
            for (int seri = 0; seri < step_size; seri++) {
                Stripe& t = stripes_.at(group[mi + seri]);
                for (auto& key : t.objects) {
                    big.objects.push_back(key);
                    std::vector<int> blocks;
                    for (int b : objects_.at(key).second) {
                        int row = -1, col = -1;
                        ecg_ec_bid2rowcol(t.ec, b, &row, &col);
                        blocks.push_back(ecg_ec_rowcol2bid(big.ec, seri * k2 + row, col));
                    }
                    objects_[key] = {big.stripe_id, blocks};
                }
                ecg_ec_destroy(t.ec);
                stripes_.erase(group[mi + seri]);
            }
            if (new_groups.empty() || (int)new_groups.back().size() == I.schema.x) new_groups.push_back({});
            new_groups.back().push_back(big.stripe_id);
            stripes_[big.stripe_id] = big;
            stats.merges++;
            stats.merged_parities += (long)cols * m2;
        }
    }
    I.merge_groups = new_groups;
    stats.merge_s += now_s() - t0;
    return all_ok;
}

std::string Loopback::mismatches_json(size_t max_entries) const {
    std::ostringstream o;
    o << "[";
    for (size_t i = 0; i < mismatches.size() && i < max_entries; i++) {
        const Mismatch& m = mismatches[i];
        o << (i ? ", " : "") << "{\"stripe\": " << m.stripe_id << ", \"failures\": [";
        for (size_t j = 0; j < m.failures.size(); j++) o << (j ? ", " : "") << m.failures[j];
        o << "], \"plans\": [";
        for (size_t j = 0; j < m.plan_kinds.size(); j++) o << (j ? ", " : "") << "\"" << m.plan_kinds[j] << "\"";
        o << "]}";
    }
    o << "]";
    return o.str();
}

std::string Loopback::manifest_json() const {
    const Impl& I = *impl_;
    std::ostringstream o;
    o << "{\"ec_type\": " << I.schema.ec_type << ", \"block_size\": " << I.schema.block_size << ", \"stripes\": [";
    bool first = true;
    for (auto& kv : stripes_) {
        const Stripe& s = kv.second;
        ecg_coding_parameters cp{};
        ecg_ec_get_coding_parameters(s.ec, &cp);
        o << (first ? "" : ", ") << "{\"id\": " << s.stripe_id << ", \"k\": " << s.k << ", \"m\": " << s.m
          << ", \"cp\": {\"k\": " << cp.k << ", \"m\": " << cp.m << ", \"l\": " << cp.l << ", \"g\": " << cp.g
          << ", \"k1\": " << cp.k1 << ", \"m1\": " << cp.m1 << ", \"k2\": " << cp.k2 << ", \"m2\": " << cp.m2
          << ", \"x\": " << cp.x << ", \"seri_num\": " << cp.seri_num << "}, \"blocks\": [";
        for (size_t i = 0; i < s.block_ids.size(); i++)
            o << (i ? ", " : "") << "[" << s.block_ids[i] << ", " << I.topo.node_port(s.blocks2nodes[i]) << "]";
        o << "], \"objects\": [";
        bool f2 = true;
        for (auto& key : s.objects) {
            o << (f2 ? "" : ", ") << "[\"" << key << "\", [";
            const auto& blocks = objects_.at(key).second;
            for (size_t j = 0; j < blocks.size(); j++) o << (j ? ", " : "") << blocks[j];
            o << "]]";
            f2 = false;
        }
        o << "]}";
        first = false;
    }
    o << "]}";
    return o.str();
}

}  // namespace ecg_loopback
