// C++ consumer of the ErasureCode facade (INTEGRATION.md Option B): the reference's proxy-side calls
// through ecg::ec_factory and the facade classes directly (csrc/codes.hpp), linked against libecg.so.
//   facade_consumer plans                 -> Azure-LRC(12,2,2): encoding matrix + repair plan for block 0 (CPU)
//   facade_consumer bytes IN OUT B        -> reads 12*B data bytes; writes the 4 parities of Azure(12,2,2)
//                                            (proxy.cpp:346 encode), then block 0 repaired by partial decoding
//                                            the way handle_repair.cpp does it (helper partial over {3,4,5},
//                                            main partial over {1,2,14} + perform_addition)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "codes.hpp"

int main(int argc, char** argv) {
    ecg::CodingParameters cp{};
    cp.k = 12;
    cp.l = 2;
    cp.g = 2;
    cp.local_or_column = 1;
    ecg::ErasureCode* ec = ecg::ec_factory(ECG_AZURE_LRC, cp);  // metadata.cpp:48-77
    if (!ec) return 2;
    ec->init_coding_parameters(cp);
    if (argc >= 2 && !strcmp(argv[1], "plans")) {
        std::vector<int> M((size_t)ec->k * ec->m);
        if (ec->make_encoding_matrix(M.data()) != 0) return 1;
        printf("matrix");
        for (int v : M) printf(" %d", v);
        printf("\n");
        ec->partition_optimal();
        std::vector<ecg::RepairPlan> plans;
        if (ec->generate_repair_plan({0}, plans) != 1) return 1;
        for (auto& p : plans) {
            printf("plan %d", (int)p.local_or_column);
            for (auto& h : p.help_blocks) {
                printf(" |");
                for (int b : h) printf(" %d", b);
            }
            printf("\n");
        }
        delete ec;
        return 0;
    }
    if (argc < 5 || strcmp(argv[1], "bytes")) return 2;
    const int B = atoi(argv[4]);
    std::vector<char> value((size_t)ec->k * B);
    FILE* f = fopen(argv[2], "rb");
    if (!f || fread(value.data(), 1, value.size(), f) != value.size()) return 2;
    fclose(f);
    std::vector<std::vector<char>> parity(ec->m, std::vector<char>(B));
    std::vector<char*> data(ec->k), coding(ec->m);
    for (int j = 0; j < ec->k; j++) data[j] = value.data() + (size_t)j * B;
    for (int j = 0; j < ec->m; j++) coding[j] = parity[j].data();
    if (ec->encode(data.data(), coding.data(), B) != 0) return 1;
    // repair block 0 from its local group {1..5, 14}: helper cluster {3,4,5}, main cluster {1,2,14}
    auto blk = [&](int b) { return b < ec->k ? data[b] : coding[b - ec->k]; };
    const std::vector<int> surv = {1, 2, 3, 4, 5, 14}, helper = {3, 4, 5}, mine = {1, 2, 14};
    std::vector<char> part_h(B), part_m(B), rebuilt(B);
    std::vector<char*> in_h = {blk(3), blk(4), blk(5)}, in_m = {blk(1), blk(2), blk(14)};
    char* out_h[1] = {part_h.data()};
    char* out_m[1] = {part_m.data()};
    if (ec->encode_partial_blocks_for_decoding(in_h.data(), out_h, B, helper, surv, {0}) != 0) return 1;
    if (ec->encode_partial_blocks_for_decoding(in_m.data(), out_m, B, mine, surv, {0}) != 0) return 1;
    char* parts[2] = {part_h.data(), part_m.data()};
    char* out[1] = {rebuilt.data()};
    if (ec->perform_addition(parts, out, B, 2, 1) != 0) return 1;
    FILE* o = fopen(argv[3], "wb");
    if (!o) return 2;
    for (auto& p : parity) fwrite(p.data(), 1, B, o);
    fwrite(rebuilt.data(), 1, B, o);
    fclose(o);
    delete ec;
    printf("ok\n");
    return 0;
}
