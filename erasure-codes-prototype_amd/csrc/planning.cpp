// Partitioning and repair planning for the ErasureCode facade.
//
// A partition is the set of a stripe's blocks placed in one cluster; a repair plan lists, per failed
// set, the blocks each cluster contributes (each inner vector becomes one partial-decoding call at a
// helper proxy, handle_repair.cpp:169-176).  Host-only integer logic, restated from the reference's
// control flow (file:line per method).  Two deliberate, documented differences:
//   * ties in the "largest partition first" orderings are broken stably (std::stable_sort); the
//     reference uses std::sort, which libstdc++ implements as a stable insertion sort for <= 16
//     elements (every BASELINE configuration) and leaves unspecified above that;
//   * random placement draws from a per-object splitmix64 stream instead of a fresh
//     random_device-seeded mt19937 per draw (utils.cpp:6-21): same support, uniform, reproducible.
#include <algorithm>
#include <random>

#include "codes.hpp"

namespace ecg {

namespace {

bool cmp_descending(const std::pair<int, int>& a, const std::pair<int, int>& b) {  // utils.cpp:159-162
    return a.second > b.second;
}

void sort_descending(std::vector<std::pair<int, int>>& v) { std::stable_sort(v.begin(), v.end(), cmp_descending); }

bool contains(const std::vector<int>& v, int x) { return std::find(v.begin(), v.end(), x) != v.end(); }

}  // namespace

// ------------------------------------------------------------------ ErasureCode

uint64_t ErasureCode::next_random() {
    if (!rng_seeded_) {
        std::random_device rd;
        rng_ = ((uint64_t)rd() << 32) ^ rd();
        rng_seeded_ = true;
    }
    uint64_t z = (rng_ += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

int ErasureCode::random_range(int lo, int hi) {  // [lo, hi], utils.cpp:15-21
    if (hi < lo) return lo;
    return lo + (int)(next_random() % (uint64_t)(hi - lo + 1));
}

int ErasureCode::random_index(int len) {  // [0, len - 1], utils.cpp:6-12
    return len <= 0 ? 0 : (int)(next_random() % (uint64_t)len);
}

void ErasureCode::partition_flat() {  // erasure_code.cpp:150-157
    for (int i = 0; i < k + m; i++) partition_plan.push_back({i});
}

int ErasureCode::generate_partition() {  // erasure_code.cpp:159-169
    partition_plan.clear();
    switch (placement_rule) {
        case ECG_PLACE_FLAT: partition_flat(); return ECG_OK;
        case ECG_PLACE_RANDOM: partition_random(); return ECG_OK;
        case ECG_PLACE_OPTIMAL: partition_optimal(); return ECG_OK;
        case ECG_PLACE_SUB_OPTIMAL: return partition_sub_optimal();
        default: return ECG_EINVAL;
    }
}

// ------------------------------------------------------------------ RS (rs.cpp:78-279)

void RSCode::partition_random() {  // rs.cpp:78-101
    const int n = k + m;
    std::vector<int> blocks(n);
    for (int i = 0; i < n; i++) blocks[i] = i;
    int cnt = 0;
    while (cnt < n) {
        const int size = std::min(random_range(1, m), n - cnt);  // single-region fault tolerance
        std::vector<int> partition;
        for (int i = 0; i < size; i++, cnt++) {
            const int at = random_index(n - cnt);
            partition.push_back(blocks[at]);
            blocks.erase(blocks.begin() + at);
        }
        partition_plan.push_back(partition);
    }
}

void RSCode::partition_optimal() {  // rs.cpp:103-116: every m consecutive blocks
    const int n = k + m;
    for (int cnt = 0; cnt < n;) {
        std::vector<int> partition;
        for (int i = 0, size = std::min(m, n - cnt); i < size; i++) partition.push_back(cnt++);
        partition_plan.push_back(partition);
    }
}

void RSCode::help_blocks_for_single_block_repair_oneoff(int failure_idx,
                                                        std::vector<std::vector<int>>& help_blocks) {
    // rs.cpp:123-180: the failed block's own partition first, then the others largest first, k in all
    const int np = (int)partition_plan.size();
    if (!np) return;
    int main_idx = -1;
    std::vector<std::pair<int, int>> others;
    for (int i = 0; i < np; i++) {
        if (contains(partition_plan[i], failure_idx)) main_idx = i;
        else others.push_back({i, (int)partition_plan[i].size()});
    }
    if (main_idx < 0) return;  // the reference indexes partition_plan[-1] here (undefined); refuse instead
    sort_descending(others);
    int cnt = 0;
    std::vector<int> main_help;
    for (int idx : partition_plan[main_idx]) {
        if (idx == failure_idx) continue;
        if (cnt < k) {
            main_help.push_back(idx);
            cnt++;
        } else {
            break;
        }
    }
    if (cnt > 0) help_blocks.push_back(main_help);
    if (cnt == k) return;
    for (auto& pr : others) {
        std::vector<int> help;
        for (int idx : partition_plan[pr.first]) {
            if (cnt < k) {
                help.push_back(idx);
                cnt++;
            } else {
                break;
            }
        }
        if (cnt > 0 && cnt <= k) help_blocks.push_back(help);
        if (cnt == k) return;
    }
}

void RSCode::help_blocks_for_multi_blocks_repair_oneoff(const std::vector<int>& failure_idxs,
                                                        std::vector<std::vector<int>>& help_blocks) {
    // rs.cpp:182-262: partitions holding failures first (largest remainder first), then the rest
    const int np = (int)partition_plan.size();
    if (!np) return;
    std::vector<std::vector<int>> part = partition_plan;
    std::vector<int> failures_cnt(np, 0);
    for (int f : failure_idxs)
        for (int i = 0; i < np; i++) {
            auto it = std::find(part[i].begin(), part[i].end(), f);
            if (it != part[i].end()) {
                failures_cnt[i]++;
                part[i].erase(it);
                break;
            }
        }
    std::vector<std::pair<int, int>> mains, others;
    for (int i = 0; i < np; i++) (failures_cnt[i] ? mains : others).push_back({i, (int)part[i].size()});
    sort_descending(mains);
    sort_descending(others);
    int cnt = 0;
    for (auto* list : {&mains, &others})
        for (auto& pr : *list) {
            std::vector<int> help;
            for (int idx : part[pr.first]) {
                if (cnt < k) {
                    help.push_back(idx);
                    cnt++;
                } else {
                    break;
                }
            }
            if (cnt > 0 && cnt <= k && !help.empty()) help_blocks.push_back(help);
            if (cnt == k) return;
        }
}

int RSCode::generate_repair_plan(const std::vector<int>& failure_idxs, std::vector<RepairPlan>& plans) {
    // rs.cpp:264-279 (no decodability check in the reference)
    if (failure_idxs.empty()) return ECG_EINVAL;
    for (int f : failure_idxs)
        if (f < 0 || f >= k + m) return ECG_EINVAL;
    RepairPlan plan;
    plan.failure_idxs = failure_idxs;
    if (failure_idxs.size() == 1) help_blocks_for_single_block_repair_oneoff(failure_idxs[0], plan.help_blocks);
    else help_blocks_for_multi_blocks_repair_oneoff(failure_idxs, plan.help_blocks);
    plans.push_back(plan);
    return 1;
}

// ------------------------------------------------------------------ LRC family (lrc.cpp)

void LocallyRepairableCode::partition_random() {  // lrc.cpp:215-238: partitions of 1..g+1 blocks
    const int n = k + l + g;
    std::vector<int> blocks(n);
    for (int i = 0; i < n; i++) blocks[i] = i;
    int cnt = 0;
    while (cnt < n) {
        const int size = std::min(random_range(1, g + 1), n - cnt);
        std::vector<int> partition;
        for (int i = 0; i < size; i++, cnt++) {
            const int at = random_index(n - cnt);
            partition.push_back(blocks[at]);
            blocks.erase(blocks.begin() + at);
        }
        partition_plan.push_back(partition);
    }
}

void LocallyRepairableCode::help_blocks_for_single_block_repair_oneoff(
        int failure_idx, std::vector<std::vector<int>>& help_blocks) {  // lrc.cpp:240-323
    const int np = (int)partition_plan.size();
    if (!np) return;
    if (local_or_column) {  // every partition contributes its members of the failed block's group
        const int gid = bid2gid(failure_idx);
        for (int i = 0; i < np; i++) {
            std::vector<int> help;
            for (int b : partition_plan[i])
                if (bid2gid(b) == gid && b != failure_idx) help.push_back(b);
            if (!help.empty()) help_blocks.push_back(help);
        }
        return;
    }
    // global repair: k survivors among data + global parities, the failed block's partition first
    int main_idx = 0;
    std::vector<std::pair<int, int>> others;
    for (int i = 0; i < np; i++) {
        int cnt = 0;
        for (int b : partition_plan[i]) {
            if (b < k + g && b != failure_idx) cnt++;
            if (b == failure_idx) {
                main_idx = i;
                cnt = 0;
                break;
            }
        }
        if (cnt > 0) others.push_back({i, cnt});
    }
    sort_descending(others);
    int cnt = 0;
    std::vector<int> main_help;
    for (int idx : partition_plan[main_idx]) {
        if (idx != failure_idx && idx < k + g) {
            if (cnt < k) {
                main_help.push_back(idx);
                cnt++;
            } else {
                break;
            }
        }
    }
    if (cnt > 0) help_blocks.push_back(main_help);
    if (cnt == k) return;
    for (auto& pr : others) {
        std::vector<int> help;
        for (int idx : partition_plan[pr.first]) {
            if (idx < k + g) {
                if (cnt < k) {
                    help.push_back(idx);
                    cnt++;
                } else {
                    break;
                }
            }
        }
        if (cnt > 0 && cnt <= k) help_blocks.push_back(help);
        if (cnt == k) return;
    }
}

void LocallyRepairableCode::help_blocks_for_multi_blocks_repair_oneoff(
        const std::vector<int>& failure_idxs, std::vector<std::vector<int>>& help_blocks) {  // lrc.cpp:325-443
    bool all_survivors = (int)failure_idxs.size() > g;
    for (int f : failure_idxs)
        if (f >= k + g) all_survivors = true;
    const int np = (int)partition_plan.size();
    if (!np) return;
    std::vector<std::vector<int>> part = partition_plan;
    if (all_survivors) {  // a local parity failed or more than g failures: every surviving block
        for (int f : failure_idxs)
            for (int i = 0; i < np; i++) {
                auto it = std::find(part[i].begin(), part[i].end(), f);
                if (it != part[i].end()) {
                    part[i].erase(it);
                    break;
                }
            }
        for (auto& p : part)
            if (!p.empty()) help_blocks.push_back(p);
        return;
    }
    // only data / global parity failures: k survivors among data + global parities
    std::vector<int> failures_cnt(np, 0);
    for (int f : failure_idxs)
        for (int i = 0; i < np; i++) {
            auto it = std::find(part[i].begin(), part[i].end(), f);
            if (it != part[i].end()) {
                failures_cnt[i]++;
                part[i].erase(it);
                break;
            }
        }
    for (int lp = k + g; lp < k + g + l; lp++)
        for (int i = 0; i < np; i++) {
            auto it = std::find(part[i].begin(), part[i].end(), lp);
            if (it != part[i].end()) {
                part[i].erase(it);
                break;
            }
        }
    std::vector<std::pair<int, int>> mains, others;
    for (int i = 0; i < np; i++) (failures_cnt[i] ? mains : others).push_back({i, (int)part[i].size()});
    sort_descending(mains);
    sort_descending(others);
    int cnt = 0;
    for (auto* list : {&mains, &others})
        for (auto& pr : *list) {
            std::vector<int> help;
            for (int idx : part[pr.first]) {
                if (cnt < k) {
                    help.push_back(idx);
                    cnt++;
                } else {
                    break;
                }
            }
            if (cnt > 0 && cnt <= k && !help.empty()) help_blocks.push_back(help);
            if (cnt == k) return;
        }
}

int LocallyRepairableCode::generate_repair_plan(const std::vector<int>& failure_idxs,
                                                std::vector<RepairPlan>& plans) {  // lrc.cpp:445-574
    const int n = k + g + l;
    if (failure_idxs.empty()) return ECG_EINVAL;
    for (int f : failure_idxs)
        if (f < 0 || f >= n) return ECG_EINVAL;
    int dec = check_if_decodable(failure_idxs);
    if (dec != 1) return dec < 0 ? dec : 0;
    if (failure_idxs.size() == 1) {
        RepairPlan plan;
        plan.failure_idxs = failure_idxs;
        local_or_column = plan.local_or_column = bid2gid(failure_idxs[0]) < l;
        help_blocks_for_single_block_repair_oneoff(failure_idxs[0], plan.help_blocks);
        plans.push_back(plan);
        return 1;
    }
    std::vector<int> failed(n, 0), group_cnt(l + 1, 0);
    int n_dg = 0, n_failed = (int)failure_idxs.size();
    for (int f : failure_idxs) {
        failed[f] = 1;
        group_cnt[bid2gid(f)] += 1;
        if (f < k + g) n_dg += 1;
    }
    for (int iter = 0; n_failed > 0; iter++) {
        for (int gid = 0; gid < l; gid++) {  // groups with one failure: local repair
            if (group_cnt[gid] != 1) continue;
            int fi = -1;
            for (int i = 0; i < n; i++)
                if (failed[i] && bid2gid(i) == gid) {
                    fi = i;
                    break;
                }
            RepairPlan plan;
            plan.local_or_column = true;
            plan.failure_idxs.push_back(fi);
            local_or_column = true;
            help_blocks_for_single_block_repair_oneoff(fi, plan.help_blocks);
            plans.push_back(plan);
            failed[fi] = 0;
            group_cnt[gid] = 0;
            n_failed -= 1;
            if (fi < k + g) n_dg -= 1;
        }
        if (n_dg > 0 && n_dg <= g) {  // 1..g data / global failures left: global repair
            RepairPlan plan;
            plan.local_or_column = false;
            for (int i = 0; i < k + g; i++)
                if (failed[i]) plan.failure_idxs.push_back(i);
            if (plan.failure_idxs.size() == 1) {
                local_or_column = false;
                help_blocks_for_single_block_repair_oneoff(plan.failure_idxs[0], plan.help_blocks);
            } else {
                help_blocks_for_multi_blocks_repair_oneoff(plan.failure_idxs, plan.help_blocks);
            }
            plans.push_back(plan);
            for (int i = 0; i < k + g; i++)
                if (failed[i]) {
                    failed[i] = 0;
                    n_failed -= 1;
                    group_cnt[bid2gid(i)] -= 1;
                }
            n_dg = 0;
        }
        if (iter > 0 && n_failed > 0) {  // repair the rest in one go (decodability re-checked on the full set)
            if (check_if_decodable(failure_idxs) != 1) return 0;
            RepairPlan plan;
            plan.local_or_column = false;
            for (int i = 0; i < n; i++)
                if (failed[i]) plan.failure_idxs.push_back(i);
            help_blocks_for_multi_blocks_repair_oneoff(plan.failure_idxs, plan.help_blocks);
            plans.push_back(plan);
            for (int i = 0; i < n; i++)
                if (failed[i]) {
                    failed[i] = 0;
                    n_failed -= 1;
                    group_cnt[bid2gid(i)] -= 1;
                }
            n_dg = 0;
        }
    }
    return 1;
}

// Azure-style optimal partition (lrc.cpp:725-814, identical for Opt_Cau_LRC at :1660-1749): cut every
// local group into partitions of g+1, merge the remainders θ at a time, then pour the g global parities
// into the partitions with free space (largest first) or give them their own partition.
static void partition_optimal_azure_style(std::vector<std::vector<int>>& plan,
                                          const std::vector<std::vector<int>>& groups, int k, int l, int g,
                                          int r) {
    std::vector<std::vector<int>> remaining;
    for (int i = 0; i < l; i++) {
        const std::vector<int>& grp = groups[i];
        const int gs = (int)grp.size();
        for (int j = 0; j < gs; j += g + 1) {
            if (j + g + 1 > gs) {
                remaining.emplace_back(grp.begin() + j, grp.end());
                break;
            }
            plan.emplace_back(grp.begin() + j, grp.begin() + j + g + 1);
        }
    }
    int theta = l;
    if ((r + 1) % (g + 1) > 1) theta = g / ((r + 1) % (g + 1) - 1);
    const int nrem = (int)remaining.size();
    for (int i = 0; i < nrem; i += theta) {
        std::vector<int> partition;
        for (int j = i; j < i + theta && j < nrem; j++)
            partition.insert(partition.end(), remaining[j].begin(), remaining[j].end());
        plan.push_back(partition);
    }
    std::vector<std::pair<int, int>> space;
    int sum_space = 0;
    for (int i = 0; i < (int)plan.size(); i++) {
        const int nb = (int)plan[i].size();
        int ngroups = 0;
        for (int b : plan[i])
            if (b >= k + g) ngroups++;
        if (ngroups == 0) ngroups = 1;
        const int left = g + ngroups - nb;
        space.push_back({i, left});
        sum_space += left;
    }
    int left_g = g, global_idx = k;
    if (sum_space >= g) {
        sort_descending(space);
        for (size_t i = 0; i < space.size() && left_g > 0; i++) {
            if (space[i].second <= 0) continue;
            int take = space[i].second;
            if (left_g >= take) {
                left_g -= take;
            } else {
                take = left_g;
                left_g = 0;
            }
            while (take--) plan[space[i].first].push_back(global_idx++);
        }
    } else {
        std::vector<int> partition;
        while (global_idx < k + g) partition.push_back(global_idx++);
        plan.push_back(partition);
    }
}

// Opt / Uni / Azure+1 style (lrc.cpp:1071-1088, 1284-1301, 2287-2304): every g+1 blocks of a group
static void partition_optimal_grouped(std::vector<std::vector<int>>& plan, const std::vector<std::vector<int>>& groups,
                                      int l, int g) {
    for (int i = 0; i < l && i < (int)groups.size(); i++) {
        const std::vector<int>& grp = groups[i];
        const int gs = (int)grp.size();
        for (int j = 0; j < gs; j += g + 1) plan.emplace_back(grp.begin() + j, grp.begin() + std::min(gs, j + g + 1));
    }
}

// Azure: local groups [data..., local parity], then the global parities as group l.
void Azu_LRC::grouping_information(std::vector<std::vector<int>>& groups) {  // lrc.cpp:706-723
    int idx = 0;
    for (int i = 0; i < l; i++) {
        std::vector<int> grp;
        for (int j = 0, gs = std::min(r, k - i * r); j < gs; j++) grp.push_back(idx++);
        grp.push_back(k + g + i);
        groups.push_back(grp);
    }
    std::vector<int> glob;
    for (int i = 0; i < g; i++) glob.push_back(idx++);
    groups.push_back(glob);
}

void Azu_LRC::partition_optimal() {
    std::vector<std::vector<int>> groups;
    grouping_information(groups);
    partition_optimal_azure_style(partition_plan, groups, k, l, g, r);
}

int Azu_LRC::partition_sub_optimal() {  // lrc.cpp:816-873: globals together in one partition
    std::vector<std::vector<int>> groups;
    grouping_information(groups);
    std::vector<std::vector<int>> remaining;
    for (int i = 0; i < l; i++) {
        const std::vector<int>& grp = groups[i];
        const int gs = (int)grp.size();
        for (int j = 0; j < gs; j += g + 1) {
            if (j + g + 1 > gs) {
                remaining.emplace_back(grp.begin() + j, grp.end());
                break;
            }
            partition_plan.emplace_back(grp.begin() + j, grp.begin() + j + g + 1);
        }
    }
    int theta = l;
    if ((r + 1) % (g + 1) > 1) theta = g / ((r + 1) % (g + 1) - 1);
    const int nrem = (int)remaining.size();
    for (int i = 0; i < nrem; i += theta) {
        std::vector<int> partition;
        for (int j = i; j < i + theta && j < nrem; j++)
            partition.insert(partition.end(), remaining[j].begin(), remaining[j].end());
        partition_plan.push_back(partition);
    }
    if (theta == nrem && !partition_plan.empty()) {
        for (int i = k; i < k + g; i++) partition_plan.back().push_back(i);
    } else {
        std::vector<int> partition;
        for (int i = k; i < k + g; i++) partition.push_back(i);
        partition_plan.push_back(partition);
    }
    return ECG_OK;
}

// Azure+1: l-1 data groups with their local parities; the last group = global parities + its local parity.
void Azu_LRC_1::grouping_information(std::vector<std::vector<int>>& groups) {  // lrc.cpp:1051-1069
    int idx = 0;
    for (int i = 0; i < l - 1; i++) {
        std::vector<int> grp;
        for (int j = 0, gs = std::min(r, k - i * r); j < gs; j++) grp.push_back(idx++);
        grp.push_back(k + g + i);
        groups.push_back(grp);
    }
    std::vector<int> last;
    for (int i = 0; i < g; i++) last.push_back(idx++);
    last.push_back(k + g + l - 1);
    groups.push_back(last);
}

void Azu_LRC_1::partition_optimal() {
    std::vector<std::vector<int>> groups;
    grouping_information(groups);
    partition_optimal_grouped(partition_plan, groups, l, g);
}

int Azu_LRC_1::check_if_decodable(const std::vector<int>& failure_idxs) {  // lrc.cpp:881-931
    std::vector<int> b2g(k + g + l, -1), fd(l, 0), slp(l, 1);
    int sgp = g, idx = 0;
    for (int i = 0; i < l; i++) {
        for (int j = 0, gs = std::min(r, k - i * r); j < gs; j++) b2g[idx++] = i;
        b2g[k + g + i] = i;
    }
    for (int b : failure_idxs) {
        if (b < 0 || b >= k + g + l) return ECG_EINVAL;
        if (b < k) fd[b2g[b]] += 1;
        else if (b < k + g) sgp -= 1;
        else slp[b - k - g] -= 1;
    }
    for (int i = 0; i < l; i++) {
        if (i < l - 1) {
            if (slp[i] && slp[i] <= fd[i]) {
                fd[i] -= slp[i];
                slp[i] = 0;
            }
        } else if (slp[i] && sgp == g - 1) {
            sgp += 1;
        }
    }
    for (int i = 0; i < l; i++) {
        if (sgp >= fd[i]) {
            sgp -= fd[i];
            fd[i] = 0;
        } else {
            return 0;
        }
    }
    return 1;
}

// Optimal LRC / Uniform Cauchy LRC: groups over data + global parities, r per group, + local parity.
static void grouping_over_data_and_globals(std::vector<std::vector<int>>& groups, int k, int l, int g, int r) {
    int idx = 0;
    for (int i = 0; i < l; i++) {
        std::vector<int> grp;
        for (int j = 0, gs = std::min(r, k + g - i * r); j < gs; j++) grp.push_back(idx++);
        grp.push_back(k + g + i);
        groups.push_back(grp);
    }
}

// lrc.cpp:1096-1166 (Opt_LRC) == lrc.cpp:2025-2095 (Uni_Cau_LRC)
static int check_decodable_mixed_groups(const std::vector<int>& failure_idxs, int k, int l, int g, int r) {
    std::vector<int> b2g(k + g + l, -1), fd(l, 0), fgp(l, 0), slp(l, 1);
    std::vector<bool> pure(l, false);
    int sgp = g, idx = 0;
    for (int i = 0; i < l; i++) {
        const int gs = std::min(r, k + g - i * r);
        for (int j = 0; j < gs; j++) {
            if (idx >= 0 && idx < k + g + l) b2g[idx] = i;
            idx++;
        }
        pure[i] = idx <= k || idx - gs >= k;
        b2g[k + g + i] = i;
    }
    for (int b : failure_idxs) {
        if (b < 0 || b >= k + g + l) return ECG_EINVAL;
        if (b < k) {
            fd[b2g[b]] += 1;
        } else if (b < k + g) {
            fgp[b2g[b]] += 1;
            sgp -= 1;
        } else {
            slp[b - k - g] -= 1;
        }
    }
    for (int i = 0; i < l; i++) {
        if (slp[i] && pure[i]) {
            if (slp[i] <= fd[i]) {
                fd[i] -= slp[i];
                slp[i] = 0;
            }
            if (slp[i] && slp[i] == fgp[i]) {
                fgp[i] -= slp[i];
                slp[i] = 0;
                sgp += 1;
            }
        } else if (slp[i] && !pure[i]) {
            if (fd[i] == 1 && !fgp[i]) {
                fd[i] -= slp[i];
                slp[i] = 0;
            } else if (fgp[i] == 1 && !fd[i]) {
                fgp[i] -= slp[i];
                slp[i] = 0;
                sgp += 1;
            }
        }
    }
    for (int i = 0; i < l; i++) {
        if (sgp >= fd[i]) {
            sgp -= fd[i];
            fd[i] = 0;
        } else {
            return 0;
        }
    }
    return 1;
}

void Opt_LRC::grouping_information(std::vector<std::vector<int>>& groups) {
    grouping_over_data_and_globals(groups, k, l, g, r);
}
void Opt_LRC::partition_optimal() {
    std::vector<std::vector<int>> groups;
    grouping_information(groups);
    partition_optimal_grouped(partition_plan, groups, l, g);
}
int Opt_LRC::check_if_decodable(const std::vector<int>& f) { return check_decodable_mixed_groups(f, k, l, g, r); }

void Uni_Cau_LRC::grouping_information(std::vector<std::vector<int>>& groups) {
    grouping_over_data_and_globals(groups, k, l, g, r);
}
void Uni_Cau_LRC::partition_optimal() {
    std::vector<std::vector<int>> groups;
    grouping_information(groups);
    partition_optimal_grouped(partition_plan, groups, l, g);
}
int Uni_Cau_LRC::check_if_decodable(const std::vector<int>& f) {
    return check_decodable_mixed_groups(f, k, l, g, r);
}

// Optimal Cauchy LRC: Azure-like groups; a local parity also covers the global parities (lrc.cpp:1485-1518).
void Opt_Cau_LRC::grouping_information(std::vector<std::vector<int>>& groups) {  // lrc.cpp:1641-1658
    int idx = 0;
    for (int i = 0; i < l; i++) {
        std::vector<int> grp;
        for (int j = 0, gs = std::min(r, k - i * r); j < gs; j++) grp.push_back(idx++);
        grp.push_back(k + g + i);
        groups.push_back(grp);
    }
    std::vector<int> glob;
    for (int i = 0; i < g; i++) glob.push_back(idx++);
    groups.push_back(glob);
}

void Opt_Cau_LRC::partition_optimal() {
    std::vector<std::vector<int>> groups;
    grouping_information(groups);
    partition_optimal_azure_style(partition_plan, groups, k, l, g, r);
}

int Opt_Cau_LRC::check_if_decodable(const std::vector<int>& failure_idxs) {  // lrc.cpp:1415-1483
    std::vector<int> b2g(k + g + l, -1), fd(l, 0), slp(l, 1);
    int fd_cnt = 0, sgp = g, idx = 0;
    for (int i = 0; i < l; i++) {
        for (int j = 0, gs = std::min(r, k - i * r); j < gs; j++) b2g[idx++] = i;
        b2g[k + g + i] = i;
    }
    for (int b : failure_idxs) {
        if (b < 0 || b >= k + g + l) return ECG_EINVAL;
        if (b < k) {
            fd[b2g[b]] += 1;
            fd_cnt += 1;
        } else if (b < k + g) {
            sgp -= 1;
        } else {
            slp[b - k - g] -= 1;
        }
    }
    if (sgp < g) {  // failed global parities are rebuilt by enough intact groups
        int healthy = 0;
        for (int i = 0; i < l; i++)
            if (slp[i] && !fd[i]) healthy++;
        if (healthy >= g - sgp) sgp = g;
    }
    if (sgp < g) return sgp >= fd_cnt ? 1 : 0;
    for (int i = 0; i < l; i++)
        if (slp[i] && slp[i] <= fd[i]) {
            fd[i] -= slp[i];
            slp[i] = 0;
        }
    for (int i = 0; i < l; i++) {
        if (sgp >= fd[i]) {
            sgp -= fd[i];
            fd[i] = 0;
        } else {
            return 0;
        }
    }
    return 1;
}

void Opt_Cau_LRC::help_blocks_for_single_block_repair_oneoff(
        int failure_idx, std::vector<std::vector<int>>& help_blocks) {  // lrc.cpp:1757-1859
    const int np = (int)partition_plan.size();
    if (!np) return;
    if (!local_or_column) {
        LocallyRepairableCode::help_blocks_for_single_block_repair_oneoff(failure_idx, help_blocks);
        return;  // the global branch is the base class's (lrc.cpp:1799-1858 == :264-322)
    }
    const bool global = failure_idx >= k && failure_idx < k + g;
    const int gid = global ? surviving_group_id : bid2gid(failure_idx);
    for (int i = 0; i < np; i++) {
        std::vector<int> help;
        for (int b : partition_plan[i]) {
            const bool is_global = b >= k && b < k + g;
            if (global ? ((is_global && b != failure_idx) || bid2gid(b) == gid)
                       : ((bid2gid(b) == gid && b != failure_idx) || is_global))
                help.push_back(b);
        }
        if (!help.empty()) help_blocks.push_back(help);
    }
}

int Opt_Cau_LRC::generate_repair_plan(const std::vector<int>& failure_idxs,
                                      std::vector<RepairPlan>& plans) {  // lrc.cpp:1861-2023
    const int n = k + g + l;
    if (failure_idxs.empty()) return ECG_EINVAL;
    for (int f : failure_idxs)
        if (f < 0 || f >= n) return ECG_EINVAL;
    int dec = check_if_decodable(failure_idxs);
    if (dec != 1) return dec < 0 ? dec : 0;
    if (failure_idxs.size() == 1) {
        RepairPlan plan;
        plan.failure_idxs = failure_idxs;
        local_or_column = plan.local_or_column = true;
        help_blocks_for_single_block_repair_oneoff(failure_idxs[0], plan.help_blocks);
        plans.push_back(plan);
        return 1;
    }
    // group l counts the global parities; a failed global parity also counts against every local group
    std::vector<int> failed(n, 0), group_cnt(l + 1, 0);
    int n_dg = 0, n_failed = (int)failure_idxs.size();
    for (int f : failure_idxs) {
        failed[f] = 1;
        group_cnt[bid2gid(f)] += 1;
        if (f < k + g) {
            n_dg += 1;
            if (f >= k)
                for (int j = 0; j < l; j++) group_cnt[j] += 1;
        }
    }
    for (int iter = 0; n_failed > 0; iter++) {
        for (int i = 0; i < n; i++) {  // a global parity rebuilt from a group with no other failure
            if (!(i >= k && i < k + g && failed[i])) continue;
            for (int j = 0; j < l; j++) {
                if (group_cnt[j] != 1) continue;
                RepairPlan plan;
                plan.local_or_column = true;
                plan.failure_idxs.push_back(i);
                local_or_column = true;
                surviving_group_id = j;
                help_blocks_for_single_block_repair_oneoff(i, plan.help_blocks);
                plans.push_back(plan);
                failed[i] = 0;
                for (int jj = 0; jj <= l; jj++) group_cnt[jj] -= 1;
                n_failed -= 1;
                n_dg -= 1;
                break;
            }
        }
        for (int gid = 0; gid < l; gid++) {
            if (group_cnt[gid] != 1) continue;
            int fi = -1;
            for (int i = 0; i < n; i++)
                if (failed[i] && bid2gid(i) == gid) {
                    fi = i;
                    break;
                }
            if (fi < 0) continue;  // the reference would index failed_map[-1] here; nothing to repair
            RepairPlan plan;
            plan.local_or_column = true;
            plan.failure_idxs.push_back(fi);
            local_or_column = true;
            help_blocks_for_single_block_repair_oneoff(fi, plan.help_blocks);
            plans.push_back(plan);
            failed[fi] = 0;
            group_cnt[gid] = 0;
            n_failed -= 1;
            if (fi < k + g) n_dg -= 1;
        }
        if (n_dg > 0 && n_dg <= g) {
            RepairPlan plan;
            plan.local_or_column = false;
            for (int i = 0; i < k + g; i++)
                if (failed[i]) plan.failure_idxs.push_back(i);
            if (plan.failure_idxs.size() == 1) {
                local_or_column = false;
                help_blocks_for_single_block_repair_oneoff(plan.failure_idxs[0], plan.help_blocks);
            } else {
                help_blocks_for_multi_blocks_repair_oneoff(plan.failure_idxs, plan.help_blocks);
            }
            plans.push_back(plan);
            for (int i = 0; i < k + g; i++)
                if (failed[i]) {
                    failed[i] = 0;
                    n_failed -= 1;
                    group_cnt[bid2gid(i)] -= 1;
                    if (i >= k)
                        for (int j = 0; j < l; j++) group_cnt[j] -= 1;
                }
            n_dg = 0;
        }
        if (iter > 0 && n_failed > 0) {
            if (check_if_decodable(failure_idxs) != 1) return 0;
            RepairPlan plan;
            plan.local_or_column = false;
            for (int i = 0; i < n; i++)
                if (failed[i]) plan.failure_idxs.push_back(i);
            help_blocks_for_multi_blocks_repair_oneoff(plan.failure_idxs, plan.help_blocks);
            plans.push_back(plan);
            for (int i = 0; i < n; i++)
                if (failed[i]) {
                    failed[i] = 0;
                    n_failed -= 1;
                    group_cnt[bid2gid(i)] -= 1;
                    if (i >= k && i < k + g)
                        for (int j = 0; j < l; j++) group_cnt[j] -= 1;
                }
            n_dg = 0;
        }
    }
    return 1;
}

// ------------------------------------------------------------------ Product codes (pc.cpp)

void ProductCode::partition_flat() {  // pc.cpp:378-388: one block per partition; rows: one column each
    row_code.partition_plan.clear();
    for (int i = 0; i < k + m; i++) partition_plan.push_back({i});
    for (int i = 0; i < k1 + m1; i++) row_code.partition_plan.push_back({i});
}

// One partition = whole columns (1..m1 of them); the row code's partition = those column indices.
// HVPC (pc.cpp:1091-1158) stores only the k2 row-parity blocks of a parity column (no globals).
static void pc_push_columns(ProductCode& pc, std::vector<int>& partition, int col, bool with_global) {
    const int rows = (col < pc.k1 || with_global) ? pc.k2 + pc.m2 : pc.k2;
    for (int row = 0; row < rows; row++) partition.push_back(pc.rowcol2bid(row, col));
}

void ProductCode::partition_random() {  // pc.cpp:390-421
    row_code.partition_plan.clear();
    const int n = k1 + m1;
    std::vector<int> columns(n);
    for (int i = 0; i < n; i++) columns[i] = i;
    int cnt = 0;
    while (cnt < n) {
        const int ncol = std::min(random_range(1, m1), n - cnt);
        std::vector<int> partition, row_partition;
        for (int i = 0; i < ncol; i++, cnt++) {
            const int at = random_index(n - cnt);
            const int col = columns[at];
            pc_push_columns(*this, partition, col, has_global());
            row_partition.push_back(col);
            columns.erase(columns.begin() + at);
        }
        partition_plan.push_back(partition);
        row_code.partition_plan.push_back(row_partition);
    }
}

void ProductCode::partition_optimal() {  // pc.cpp:423-443: every m1 consecutive columns
    row_code.partition_plan.clear();
    const int n = k1 + m1;
    for (int cnt = 0; cnt < n;) {
        std::vector<int> partition, row_partition;
        for (int i = 0, ncol = std::min(m1, n - cnt); i < ncol; i++, cnt++) {
            pc_push_columns(*this, partition, cnt, has_global());
            row_partition.push_back(cnt);
        }
        partition_plan.push_back(partition);
        row_code.partition_plan.push_back(row_partition);
    }
}

void HVPC::partition_random() { ProductCode::partition_random(); }
void HVPC::partition_optimal() { ProductCode::partition_optimal(); }

int ProductCode::generate_repair_plan(const std::vector<int>& failure_idxs,
                                      std::vector<RepairPlan>& plans) {  // pc.cpp:451-551, HVPC :1166-1264
    const int rows_all = k2 + m2, cols_all = k1 + m1;
    const int ncols = has_global() ? cols_all : k1, nrows = has_global() ? rows_all : k2;
    int failed_num = (int)failure_idxs.size();
    if (failed_num == 0) return ECG_EINVAL;
    std::vector<std::vector<int>> fmap(rows_all, std::vector<int>(cols_all, 0));
    std::vector<int> frc(rows_all, 0), fcc(cols_all, 0);
    for (int b : failure_idxs) {
        if (b < 0 || b >= k + m) return ECG_EINVAL;
        int r, c;
        bid2rowcol(b, r, c);
        fmap[r][c] = 1;
        frc[r]++;
        fcc[c]++;
    }
    while (failed_num > 0) {
        for (int i = 0; i < ncols; i++) {  // columns with <= m2 failures
            if (!(fcc[i] > 0 && fcc[i] <= m2)) continue;
            RepairPlan plan;
            plan.local_or_column = true;
            std::vector<int> help;
            for (int jj = 0, cnt = 0; jj < rows_all && cnt < k2; jj++)
                if (!fmap[jj][i]) {
                    help.push_back(rowcol2bid(jj, i));
                    cnt++;
                }
            if (placement_rule == ECG_PLACE_FLAT) {
                for (int b : help) plan.help_blocks.push_back({b});
            } else {
                plan.help_blocks.push_back(help);
            }
            for (int jj = 0; jj < rows_all; jj++)
                if (fmap[jj][i]) {
                    plan.failure_idxs.push_back(rowcol2bid(jj, i));
                    fmap[jj][i] = 0;
                    failed_num--;
                    frc[jj]--;
                    fcc[i]--;
                }
            plans.push_back(plan);
        }
        if (failed_num == 0) break;
        int max_row = -1;
        for (int i = 0; i < nrows; i++) {  // the first row with <= m1 failures
            if (!(frc[i] > 0 && frc[i] <= m1)) continue;
            max_row = i;
            RepairPlan plan;
            plan.local_or_column = false;
            std::vector<int> cols;
            for (int jj = 0; jj < cols_all; jj++)
                if (fmap[i][jj]) cols.push_back(jj);
            row_code.help_blocks_for_multi_blocks_repair_oneoff(cols, plan.help_blocks);
            for (auto& hb : plan.help_blocks)
                for (int& c : hb) c = rowcol2bid(i, c);
            for (int jj = 0; jj < cols_all; jj++)
                if (fmap[i][jj]) {
                    plan.failure_idxs.push_back(rowcol2bid(i, jj));
                    fmap[i][jj] = 0;
                    failed_num--;
                    frc[i]--;
                    fcc[jj]--;
                }
            plans.push_back(plan);
            break;
        }
        if (max_row == -1) return 0;
    }
    return 1;
}

}  // namespace ecg
