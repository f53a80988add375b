// Loopback harness for BASELINE config 1: coordinator-lite + proxy-lite + datanode
// block stores in one process, reproducing run_client's call sequence (project/src/client/run_client.cpp
// :147-225) through the ErasureCode C ABI (include/ecg.h), i.e. the byte work runs on the GPU engine.
//
// What is kept from the reference: placement of each partition in its own cluster (placement.cpp:77-140,
// multistripe rule RAND), repair planning by the code object (generate_repair_plan over the partitions
// found from the actual placement, auxs.cpp:139-159), concrete main/help plans (repair.cpp:190-470),
// the proxies' partial-decoding data path (handle_repair.cpp:5-470, 472-650) with the reference's wire
// framing between helper and main proxy, RS stripe merging by partial encoding (merge.cpp:19-450,
// handle_merge.cpp:5-538) and GET by reading the data blocks (proxy.cpp:428+).
// What is dropped: RPC / sockets / threads per block (control plane), cross-cluster simulation timers,
// block relocation after merging (merge.cpp:133-260 moves blocks between nodes; no byte math).
// What is stricter: failed blocks are really removed from the store before a repair and the stripe's
// metadata follows the rebuilt copies, so a plan that read a lost block would fail; every rebuilt block
// is compared with the lost original.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ecg.h"
#include "block_store.hpp"

namespace ecg_loopback {

struct Topology {  // project/clusterinfo.xml: 10 clusters x 12 datanodes
    int clusters = 10;
    int nodes_per_cluster = 12;
    int proxy_port(int c) const { return 50005 + 30 * c; }
    int node_port(unsigned node) const { return 17600 + (int)node; }
    int cluster_of(unsigned node) const { return (int)node / nodes_per_cluster; }
};

struct EcSchema {  // config.ini [ECSCHEMA] (metadata.h:33-46)
    int ec_type = ECG_RS;
    ecg_coding_parameters cp{};
    int placement_rule = ECG_PLACE_OPTIMAL;
    bool partial_decoding = true;
    size_t block_size = 1024;
    int x = 2;
};

struct Stripe {
    unsigned stripe_id = 0;
    ecg_ec* ec = nullptr;
    int k = 0, m = 0;
    std::vector<unsigned> block_ids;
    std::vector<unsigned> blocks2nodes;
    std::vector<std::string> objects;
};

struct Stats {
    long sets = 0, gets = 0, get_mismatch = 0, degraded_gets = 0;
    long repairs = 0, repairs_failed = 0, repairs_skipped_undecodable = 0, repair_plans = 0, plans_partial = 0, plans_direct = 0;
    long blocks_rebuilt = 0, rebuilt_mismatch = 0;
    long helper_messages = 0, helper_bytes = 0;
    long merges = 0, merged_parities = 0;
    long ecg_errors = 0, decode_undecodable = 0;
    double set_s = 0, repair_s = 0, merge_s = 0, get_s = 0;
};

// A repair whose rebuilt bytes differ from the lost block: the pattern and how each plan ran
// ("partial-local", "partial-global", "direct-local", "direct-global").
struct Mismatch {
    unsigned stripe_id;
    std::vector<int> failures;
    std::vector<std::string> plan_kinds;
};

class Loopback {
public:
    Loopback(const EcSchema& schema, const Topology& topo, BlockStore& store, uint64_t seed);
    ~Loopback();

    // client.set (proxy.cpp:274-427): one stripe per object of k * block_size bytes
    bool set(const std::string& key, const std::vector<char>& value);
    // client.get (proxy.cpp:428-724): the object's data blocks, concatenated; a data block whose datanode
    // does not answer is rebuilt by the degraded read (proxy.cpp:517-666)
    bool get(const std::string& key, std::vector<char>& value);
    // get() while the datanode of the object's data block `data_pos` is unreachable (block restored after)
    bool get_with_unreachable(const std::string& key, int data_pos, std::vector<char>& value);
    // client.blocks_repair (repair.cpp:5-155): returns false if the code cannot repair the set
    bool repair(unsigned stripe_id, const std::vector<int>& failures);
    // client.merge: RS, Azure LRC, PC / HVPC / HPC (horizontal), as do_stripe_merge dispatches them
    bool merge(int step_size);

    std::vector<unsigned> list_stripes() const;
    const Stripe& stripe(unsigned id) const { return stripes_.at(id); }
    int block_num(unsigned id) const { return stripes_.at(id).k + stripes_.at(id).m; }
    Stats stats;
    std::vector<Mismatch> mismatches;
    std::string manifest_json() const;
    std::string mismatches_json(size_t max_entries = 64) const;

private:
    struct Impl;
    std::unique_ptr<Impl> impl_;
    std::map<unsigned, Stripe> stripes_;
    // key -> (stripe, the object's data blocks in value order)
    std::unordered_map<std::string, std::pair<unsigned, std::vector<int>>> objects_;
    bool rs_merge(int step_size);
    bool pc_merge(int step_size);   // PC / HVPC (merge.cpp:877-1505), horizontal
    bool hpc_merge(int step_size);  // HPC (merge.cpp:1505-1905), vertical
    bool lrc_merge(int step_size);  // Azure LRC (merge.cpp:451-877)
    friend struct Impl;
};

}  // namespace ecg_loopback
