// Host cost of the per-stripe facade path (TOOL, not product): the families workload's RS(12,4) / Azure-LRC(12,2,2)
// repairs and encodes issued through loopback/replay.cpp's ecg_replay_calls in one batch scope per batch, against
// tests/tsan/hip_stub.cpp in no-op mode (HIP_STUB_NOOP=1: launches return at once), so the time measured is the
// library's own host work per recorded call: the facade, recording, scratch composition, scheduling, pointer
// tables.  tools/host_cost.sh builds it (optionally with -pg for gprof).
// usage: host_cost [batches=200] [stripes=256]
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ecg.h"

extern "C" int ecg_replay_calls(ecg_ec** handles, int n_handles, int scope_stripes, int use_scratch, char* base,
                                long long sstride, long long bstride, int B, int S, const int* pattern_of,
                                const int* prog, const int* off, int nb, int nscr, char* scratch, void* stream);

static void call(std::vector<int>& v, int kind, int h, const std::vector<int>& in, const std::vector<int>& out,
                 const std::vector<int>& a = {}, const std::vector<int>& b = {}, const std::vector<int>& c = {}) {
    v.push_back(kind);
    v.push_back(h);
    for (const auto* x : {&in, &out, &a, &b, &c}) {
        v.push_back((int)x->size());
        v.insert(v.end(), x->begin(), x->end());
    }
}

// ecg_ec_generate_repair_plan's serialisation: [n_plans, (local, nf, fails.., n_help, (size, ids..)*)*]
static void repair_prog(ecg_ec* planner, int f, int nb, std::vector<int>& prog, int& nscr) {
    int buf[4096], dec = 0;
    const int n = ecg_ec_generate_repair_plan(planner, &f, 1, buf, 4096, &dec);
    if (n <= 0 || !dec) abort();
    int at = 1, slot = nb;
    for (int p = 0; p < buf[0]; p++) {
        const int local = buf[at], nf = buf[at + 1];
        std::vector<int> fails(buf + at + 2, buf + at + 2 + nf);
        at += 2 + nf;
        const int ng = buf[at++];
        std::vector<std::vector<int>> groups;
        std::vector<int> surv, parts;
        for (int g = 0; g < ng; g++) {
            const int sz = buf[at++];
            groups.emplace_back(buf + at, buf + at + sz);
            surv.insert(surv.end(), buf + at, buf + at + sz);
            at += sz;
        }
        for (auto& grp : groups) {
            std::vector<int> outs;
            for (int u = 0; u < nf; u++) outs.push_back(slot++);
            call(prog, 1, local, grp, outs, grp, surv, fails);
            parts.insert(parts.end(), outs.begin(), outs.end());
        }
        call(prog, 2, local, parts, fails, {(int)parts.size(), nf});
    }
    nscr = std::max(nscr, slot - nb);
}

int main(int argc, char** argv) {
    const int batches = argc > 1 ? atoi(argv[1]) : 200, S = argc > 2 ? atoi(argv[2]) : 256;
    const int B = 4096;  // the stub does no byte work: the block size only sizes the arena
    struct Code {
        const char* name;
        int type;
        ecg_coding_parameters cp;
    } codes[] = {{"RS(12,4)", ECG_RS, {12, 4, 0, 0, 0, 0, 0, 0, 0, 0, 0}},
                 {"Azure_LRC(12,2,2)", ECG_AZURE_LRC, {12, 4, 2, 2, 0, 0, 0, 0, 0, 0, 0}},
                 {"PC(4,1,4,1)", ECG_PC, {0, 0, 0, 0, 4, 1, 4, 1, 0, 0, 0}}};
    for (const Code& c : codes) {
        ecg_coding_parameters cl = c.cp;
        cl.local_or_column = 1;
        ecg_ec* h[2] = {ecg_ec_factory(c.type, &c.cp), ecg_ec_factory(c.type, &cl)};
        ecg_ec* planner = ecg_ec_factory(c.type, &c.cp);
        ecg_ec_init_coding_parameters(h[0], &c.cp);
        ecg_ec_init_coding_parameters(h[1], &cl);
        ecg_ec_init_coding_parameters(planner, &c.cp);
        ecg_ec_generate_partition(planner);
        const int k = ecg_ec_k(h[0]), m = ecg_ec_m(h[0]), n = k + m;
        for (int op = 0; op < 2; op++) {
            std::vector<int> prog, off{0}, pat((size_t)S);
            int nscr = 0;
            if (op == 0) {
                std::vector<int> in, out;
                for (int j = 0; j < k; j++) in.push_back(j);
                for (int j = 0; j < m; j++) out.push_back(k + j);
                call(prog, 0, 0, in, out);
                off.push_back((int)prog.size());
            } else {
                for (int f = 0; f < n; f++) {
                    repair_prog(planner, f, n, prog, nscr);
                    off.push_back((int)prog.size());
                }
                for (int s = 0; s < S; s++) pat[s] = s % n;
            }
            char *base = nullptr, *scr = nullptr;
            hipMalloc((void**)&base, (size_t)S * n * B);
            hipMalloc((void**)&scr, (size_t)S * std::max(1, nscr) * B);
            long long calls = 0;
            double sec = 1e30;  // the best of five runs of `batches` batches (a shared CPU is noisy)
            for (int rep = 0; rep < 5; rep++) {
                auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < batches; i++) {
                    const int rc = ecg_replay_calls(h, 2, S, 1, base, (long long)n * B, B, B, S,
                                                    op ? pat.data() : nullptr, prog.data(), off.data(), n, nscr, scr,
                                                    nullptr);
                    if (rc) {
                        fprintf(stderr, "%s op %d: rc %d\n", c.name, op, rc);
                        return 1;
                    }
                }
                sec = std::min(sec, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            }
            long long rec = 0, comp = 0, launches = 0, mat = 0;
            ecg_batch_last_stats(&rec, &comp, &launches, &mat);
            calls = rec;
            printf("%-20s %-8s %4d stripes: %.1f us per batch, %lld calls per scope -> %.3f us per call (launches %lld)\n",
                   c.name, op ? "repair1" : "encode", S, sec / batches * 1e6, calls, sec / batches * 1e6 / calls, launches);
            hipFree(base);
            hipFree(scr);
        }
        ecg_ec_destroy(h[0]);
        ecg_ec_destroy(h[1]);
        ecg_ec_destroy(planner);
    }
    return 0;
}
