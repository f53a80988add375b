// ecg_loopback: run_client's sequence (project/src/client/run_client.cpp:147-225) against the loopback
// harness.  Defaults are BASELINE config 1 / project/config.ini: RS(6,4), 1 KiB blocks, OPTIMAL placement,
// partial decoding, x = 2, 64 stripes.
//
//   set every object -> single-block repair of every block of every stripe -> 5 multi-block repairs
//   (2..4 random failures) per stripe -> merge x stripes -> the same repairs on the merged stripes ->
//   degraded reads (one data block's datanode unreachable) of --degraded objects -> get every object
//   and compare.
//
// Objects are splitmix64 bytes (word w of object j = splitmix64(seed + (j*k*B/8 + w) * golden)) instead
// of the reference's one-character values (utils.cpp:92), which would hide multiply errors.
// Prints one JSON line of counters; --manifest writes the final stripe table for an external checker.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "loopback.hpp"

using namespace ecg_loopback;

namespace {

uint64_t splitmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

std::vector<char> object_bytes(uint64_t seed, uint64_t word_offset, size_t n) {
    std::vector<char> v(n);
    for (size_t w = 0; w * 8 < n; w++) {
        const uint64_t x = splitmix(seed + (word_offset + w) * 0x9E3779B97F4A7C15ULL);
        memcpy(v.data() + w * 8, &x, std::min<size_t>(8, n - w * 8));
    }
    return v;
}

int type_of(const std::string& s) {
    const char* names[] = {"RS", "ERS", "AZURE_LRC", "AZURE_LRC_1", "OPTIMAL_LRC", "OPTIMAL_CAUCHY_LRC",
                           "UNIFORM_CAUCHY_LRC", "PC", "Hierachical_PC", "HV_PC"};
    for (int i = 0; i < 10; i++)
        if (s == names[i]) return i;
    return -1;
}

int rule_of(const std::string& s) {
    if (s == "FLAT") return ECG_PLACE_FLAT;
    if (s == "RANDOM") return ECG_PLACE_RANDOM;
    if (s == "OPTIMAL") return ECG_PLACE_OPTIMAL;
    return -1;
}

// --selftest-store: the block stores alone (no GPU): store / access / overwrite / remove / batch / count
int selftest_store(const std::string& kind, const std::string& dir) {
    auto st = make_block_store(kind, dir);
    if (!st) return 2;
    const size_t B = 4096;
    std::vector<int> ports;
    std::vector<std::string> keys;
    std::vector<char> staging(16 * B), back(16 * B);
    for (int i = 0; i < 16; i++) {
        ports.push_back(17600 + i % 5);
        keys.push_back(std::to_string(1000 + i));
    }
    std::vector<char> v = object_bytes(3, 0, staging.size());
    memcpy(staging.data(), v.data(), v.size());
    int fails = 0;
    fails += !st->store_batch(ports, keys, staging.data(), B);
    fails += st->count() != 16;
    fails += !st->access_batch(ports, keys, back.data(), B);
    fails += staging != back;
    std::vector<char> one(B, 7), got(B);
    fails += !st->store_data(17600, keys[0], one.data(), B);  // overwrite
    fails += !st->access_data(17600, keys[0], got.data(), B) || got != one;
    fails += st->access_data(17601, keys[0], got.data(), B);  // other datanode: absent
    fails += !st->remove_data(17600, keys[0]);
    fails += st->access_data(17600, keys[0], got.data(), B);
    fails += st->count() != 15;
    for (int i = 1; i < 16; i++) fails += !st->remove_data(ports[i], keys[i]);
    fails += st->count() != 0;
    printf("{\"selftest_store\": \"%s\", \"failures\": %d}\n", kind.c_str(), fails);
    return fails ? 1 : 0;
}

void usage() {
    fprintf(stderr,
            "ecg_loopback [--ec RS] [--k 6 --m 4 | --k --l --g | --k1 --m1 --k2 --m2] [--block-size 1024]\n"
            "             [--stripes 64] [--x 2] [--placement OPTIMAL] [--partial 1] [--store kv|disk]\n"
            "             [--dir ./storage] [--seed 1] [--multi 5] [--degraded 8] [--no-merge] [--manifest path]\n");
}

}  // namespace

int main(int argc, char** argv) {
    EcSchema schema;
    schema.cp.k = 6;
    schema.cp.m = 4;
    int stripes = 64, multi = 5, degraded = 8;
    bool do_merge = true;
    std::string store_kind = "kv", dir = "./storage", manifest;
    uint64_t seed = 1;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto val = [&]() -> std::string {
            if (i + 1 >= argc) {
                usage();
                exit(2);
            }
            return argv[++i];
        };
        if (a == "--ec") schema.ec_type = type_of(val());
        else if (a == "--k") schema.cp.k = atoi(val().c_str());
        else if (a == "--m") schema.cp.m = atoi(val().c_str());
        else if (a == "--l") schema.cp.l = atoi(val().c_str());
        else if (a == "--g") schema.cp.g = atoi(val().c_str());
        else if (a == "--k1") schema.cp.k1 = atoi(val().c_str());
        else if (a == "--m1") schema.cp.m1 = atoi(val().c_str());
        else if (a == "--k2") schema.cp.k2 = atoi(val().c_str());
        else if (a == "--m2") schema.cp.m2 = atoi(val().c_str());
        else if (a == "--block-size") schema.block_size = (size_t)atol(val().c_str());
        else if (a == "--stripes") stripes = atoi(val().c_str());
        else if (a == "--x") schema.x = atoi(val().c_str());
        else if (a == "--placement") schema.placement_rule = rule_of(val());
        else if (a == "--partial") schema.partial_decoding = atoi(val().c_str()) != 0;
        else if (a == "--store") store_kind = val();
        else if (a == "--dir") dir = val();
        else if (a == "--seed") seed = strtoull(val().c_str(), nullptr, 0);
        else if (a == "--multi") multi = atoi(val().c_str());
        else if (a == "--degraded") degraded = atoi(val().c_str());
        else if (a == "--no-merge") do_merge = false;
        else if (a == "--manifest") manifest = val();
        else if (a == "--selftest-store") return selftest_store(store_kind, dir);
        else {
            usage();
            return 2;
        }
    }
    if (schema.ec_type < 0 || schema.placement_rule < 0 || schema.block_size % 8 != 0 || stripes < 1) {
        usage();
        return 2;
    }
    // LRC / PC parameter conventions of config.ini: m is derived by the code
    if (schema.ec_type >= ECG_AZURE_LRC && schema.ec_type <= ECG_UNIFORM_CAUCHY_LRC) schema.cp.m = schema.cp.l + schema.cp.g;
    if (schema.ec_type >= ECG_PC) schema.cp.k = schema.cp.k1 * schema.cp.k2;
    auto store = make_block_store(store_kind, dir);
    if (!store) {
        usage();
        return 2;
    }
    Topology topo;
    Loopback lb(schema, topo, *store, seed);
    std::mt19937_64 rng(seed ^ 0x5eedULL);

    // set
    const size_t value_len = (size_t)schema.cp.k * schema.block_size;
    std::vector<std::string> keys;
    for (int j = 0; j < stripes; j++) {
        char key[32];
        snprintf(key, sizeof(key), "obj%05d", j);
        keys.push_back(key);
        if (!lb.set(key, object_bytes(seed, (uint64_t)j * value_len / 8, value_len))) {
            fprintf(stderr, "set %s failed\n", key);
            return 1;
        }
    }
    auto repairs = [&](long& singles, long& multis) {
        for (unsigned sid : lb.list_stripes()) {  // test_single_block_repair (run_client.cpp:6-56)
            const int n = lb.block_num(sid);
            for (int j = 0; j < n; j++) singles += lb.repair(sid, {j});
        }
        for (unsigned sid : lb.list_stripes()) {  // test_multiple_blocks_repair (run_client.cpp:58-108)
            const int n = lb.block_num(sid);
            for (int r = 0; r < multi; r++) {
                const int nf = 2 + (int)(rng() % 3);  // random_range(2, 4)
                std::set<int> f;
                while ((int)f.size() < std::min(nf, n)) f.insert((int)(rng() % n));
                multis += lb.repair(sid, std::vector<int>(f.begin(), f.end()));
            }
        }
    };
    long pre_single = 0, pre_multi = 0, post_single = 0, post_multi = 0;
    repairs(pre_single, pre_multi);
    bool merged = false;
    const bool mergeable = schema.ec_type == ECG_RS || schema.ec_type == ECG_AZURE_LRC || schema.ec_type >= ECG_PC;
    if (do_merge && mergeable) {
        merged = lb.merge(schema.x);
        // A merged HPC stripe's rows are RS(x*k1, m1) while the coordinator keeps addressing them as
        // ERS(k1', m1, x, seri) (repair.cpp:393-409), so post-merge HPC repairs would use the wrong
        // matrix in the reference; they are not run.
        if (schema.ec_type != ECG_HIERACHICAL_PC) repairs(post_single, post_multi);
    }
    // degraded reads (proxy.cpp:517-666): the datanode of one random data block of an object does not
    // answer; the GET rebuilds it through ec->decode
    long degraded_ok = 0, degraded_tried = 0;
    for (int j = 0; j < std::min(degraded, (int)keys.size()); j++) {
        std::vector<char> v;
        const int pos = (int)(rng() % schema.cp.k);
        degraded_tried++;
        if (lb.get_with_unreachable(keys[j], pos, v) && v == object_bytes(seed, (uint64_t)j * value_len / 8, value_len))
            degraded_ok++;
    }
    // get
    long get_ok = 0;
    for (size_t j = 0; j < keys.size(); j++) {
        std::vector<char> v;
        if (lb.get(keys[j], v) && v == object_bytes(seed, (uint64_t)j * value_len / 8, value_len)) get_ok++;
        else lb.stats.get_mismatch++;
    }
    if (!manifest.empty()) {
        std::ofstream(manifest) << lb.manifest_json() << "\n";
    }
    const Stats& s = lb.stats;
    long long worker_calls = 0;  // small calls the resident call worker took (ECG_CALL_WORKER)
    (void)ecg_call_worker_stats(&worker_calls, nullptr, nullptr, nullptr);
    printf("{\"ec_type\": %d, \"k\": %d, \"m\": %d, \"block_size\": %zu, \"stripes\": %d, \"store\": \"%s\", "
           "\"partial_decoding\": %s, \"sets\": %ld, \"repairs\": %ld, \"repairs_ok_pre_merge\": [%ld, %ld], "
           "\"repairs_ok_post_merge\": [%ld, %ld], \"repairs_failed\": %ld, \"skipped_undecodable\": %ld, "
           "\"repair_plans\": %ld, "
           "\"plans_partial\": %ld, \"plans_direct\": %ld, \"blocks_rebuilt\": %ld, \"rebuilt_mismatch\": %ld, "
           "\"helper_messages\": %ld, \"helper_bytes\": %ld, \"merged\": %s, \"merges\": %ld, "
           "\"merged_parities\": %ld, \"final_stripes\": %zu, \"gets_ok\": %ld, \"get_mismatch\": %ld, "
           "\"degraded_gets\": %ld, \"degraded_ok\": %ld, "
           "\"ecg_errors\": %ld, \"decode_undecodable\": %ld, \"blocks_in_store\": %zu, \"seconds\": {\"set\": %.4f, \"repair\": %.4f, "
           "\"merge\": %.4f, \"get\": %.4f}, \"call_worker_calls\": %lld, \"mismatches\": %s}\n",
           schema.ec_type, schema.cp.k, schema.cp.m, schema.block_size, stripes, store_kind.c_str(),
           schema.partial_decoding ? "true" : "false", s.sets, s.repairs, pre_single, pre_multi, post_single,
           post_multi, s.repairs_failed, s.repairs_skipped_undecodable, s.repair_plans, s.plans_partial, s.plans_direct,
           s.blocks_rebuilt, s.rebuilt_mismatch, s.helper_messages, s.helper_bytes, merged ? "true" : "false",
           s.merges, s.merged_parities, lb.list_stripes().size(), get_ok, s.get_mismatch, degraded_tried, degraded_ok,
           s.ecg_errors,
           s.decode_undecodable, store->count(), s.set_s, s.repair_s, s.merge_s, s.get_s, worker_calls,
           lb.mismatches_json().c_str());
    // exit status: 0 = every repair rebuilt the lost bytes; mismatches are listed for the checker
    const bool pass = s.rebuilt_mismatch == 0 && s.get_mismatch == 0 && s.ecg_errors == 0 &&
                      s.repairs_failed == s.decode_undecodable &&
                      get_ok == (long)keys.size();
    return pass ? 0 : 1;
}
