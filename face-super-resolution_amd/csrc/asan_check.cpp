// Host-side AddressSanitizer check of the C-ABI ("Race detection /
// sanitizers"): `make asan` builds libfen_hip with the HOST half of every HIP source
// instrumented (-Xarch_host -fsanitize=address; device code is untouched) and this driver,
// linked with the ASan runtime, calls every host path of include/fen.h that runs without a GPU:
// the pure queries, each entry point's argument validation, the multi-job table builders
// (fen_pack_table, fen_wgrad_multi_work_floats), the chained group launch's descriptor checks,
// table build and hash (fen_group_strip_chain_prepare up to its launch), the status word
// exchange and the RCCL entry points' refusals and library resolution.  Any heap / stack
// overflow, use-after-free or leak in those paths aborts the run with an ASan report; a wrong
// return code fails an expectation.  Not product code: nothing links it but the asan target.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fen.h"

static int g_fail = 0;
#define EXPECT(c)                                                          \
    do {                                                                   \
        if (!(c)) {                                                        \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                      \
        }                                                                  \
    } while (0)

static void* fake(size_t i) { return (void*)(uintptr_t)(0x10000 * (i + 1)); }

static void pure_queries() {
    for (int c = -8; c <= 1; ++c) EXPECT(fen_status_string(c) != nullptr && std::strlen(fen_status_string(c)) > 0);
    EXPECT(std::strstr(fen_build_info(), "gfx950") != nullptr);
    EXPECT(fen_last_hip_error() != nullptr);
    EXPECT(fen_packed_elems(0, 3, 64) == 9 * 16 * 64);
    EXPECT(fen_packed_elems(2, 256, 64) == 9 * 64 * 256);
    EXPECT(fen_pool_parts(4096) == 64);
    EXPECT(fen_sumsq_parts(5115651) == 1024);
    EXPECT(fen_feat_loss_parts() > 0);
    EXPECT(fen_ssim_parts(2, 3, 64, 64) > 0 && fen_ssim_work_floats(2, 3, 64, 64) == (size_t)3 * 2 * 3 * 64 * 64);
    EXPECT(fen_bn_work_floats(64) > 0);
    {   // grouped BN refusals (host checks only: no launch)
        float f = 0.f;
        EXPECT(fen_bn_stats_n(FEN_BF16, 0, 16, 64, &f, 1e-5f, 0.1f, &f, nullptr, nullptr, &f, nullptr) == FEN_EINVAL);
        EXPECT(fen_bn_stats_n(FEN_BF16, 2, 16, 60, &f, 1e-5f, 0.1f, &f, nullptr, nullptr, &f, nullptr) == FEN_EINVAL);
        EXPECT(fen_bn_stats_n(FEN_BF16, 2, 16, 64, &f, 1e-5f, 0.1f, &f, &f, nullptr, &f, nullptr) == FEN_EINVAL);
        EXPECT(fen_bn_apply_n(FEN_BF16, 2, 16, 64, &f, &f, &f, 32, &f, &f, 0.2f, &f, nullptr) == FEN_EINVAL);
        EXPECT(fen_bn_apply_n(FEN_BF16, 1, 16, 2048, &f, &f, &f, 0, &f, &f, 0.2f, &f, nullptr) == FEN_EUNSUPPORTED);
        EXPECT(fen_bn_bwd_n(FEN_BF16, 0, 16, 64, &f, &f, &f, &f, &f, 0.2f, &f, &f, &f, 0, &f, nullptr) == FEN_EINVAL);
        EXPECT(fen_bn_bwd_n(FEN_BF16, 2, 16, 64, &f, &f, &f, &f, &f, 0.2f, &f, &f, &f, 0, nullptr, nullptr) == FEN_EINVAL);
    }
    EXPECT(fen_conv_first_work_floats(2, 3, 64, 64, 64) > 0);
    EXPECT(fen_conv_last_dgrad_part_rows(2, 256, 256) > 0);
    EXPECT(fen_group_strip_work_bytes(32, 64) > 0 && fen_group_strip_bwd_work_bytes(32, 64) > 0);
    EXPECT(fen_group_strip_bwd_dal_rows(32, 64) > 0);
    EXPECT(fen_rcab_c128_tiles(128, 128) > 0);
    EXPECT(fen_group_strip_supported(FEN_BF16, 32, 64, 64, 64, 16, 10) == 1);
    EXPECT(fen_group_strip_supported(FEN_F32, 32, 64, 64, 64, 16, 10) == 0);
    EXPECT(fen_rcab_deferred_supported(FEN_BF16, 32, 64, 64, 64, 16) == 1);
    EXPECT(fen_rcab_deferred_supported(FEN_BF16, 32, 64, 64, 128, 32) == 0);
}

static void conv_refusals() {
    EXPECT(fen_conv3x3(nullptr, nullptr) == FEN_EINVAL);
    fen_conv_desc d;
    std::memset(&d, 0, sizeof d);
    d.dtype = FEN_BF16, d.B = 1, d.H = 8, d.W = 8, d.Cin = 36, d.Cout = 64;   // 72-B rows
    d.x = d.w = d.y = fake(0);
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EUNSUPPORTED);
    d.Cin = 64;
    d.epi = FEN_EPI_DOT;
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EINVAL);                      // no pre_in / part
    d.pre_in = fake(1), d.part = (float*)fake(2);
    d.epi = FEN_EPI_DOT | FEN_EPI_POOL;
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EUNSUPPORTED);
    d.epi = FEN_EPI_SHUFFLE | FEN_EPI_UNSHUFFLE;
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EUNSUPPORTED);
    d.epi = 0, d.s2d_in = 48;
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EINVAL);
    d.s2d_in = 0, d.dtype = 7;
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EINVAL);
    d.dtype = FEN_BF16, d.pre_in = nullptr, d.part = nullptr;
    d.epi = FEN_EPI_RELU_BWD;
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EINVAL);                      // no pre_in
    d.pre_in = fake(1), d.part = (float*)fake(2);
    d.epi = FEN_EPI_RELU_BWD | FEN_EPI_PRELU_BWD;
    d.alpha = (const float*)fake(3);
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EUNSUPPORTED);
    d.epi = 1 << 20;
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EINVAL);                      // unknown flag
    d.epi = 0, d.y_images = 1;
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EINVAL);                      // y_images without y_pool
    d.y_images = 0, d.y_pool = fake(4);
    EXPECT(fen_conv3x3(&d, nullptr) == FEN_EUNSUPPORTED);                // y_pool without PReLU
}

static void wgrad_tables() {
    std::vector<fen_wgrad_desc> a(FEN_WGRAD_MAXJOBS + 1);
    for (auto& d : a) {
        std::memset(&d, 0, sizeof d);
        d.dtype = FEN_BF16, d.B = 32, d.H = 64, d.W = 64, d.Cin = 64, d.Cout = 64, d.cout_valid = 64;
        d.x = d.dy = fake(0), d.dw = (float*)fake(1), d.work = (float*)fake(2);
    }
    EXPECT(fen_wgrad3x3_multi(0, a.data(), nullptr) == FEN_EINVAL);
    EXPECT(fen_wgrad3x3_multi(FEN_WGRAD_MAXJOBS + 1, a.data(), nullptr) == FEN_EINVAL);
    EXPECT(fen_wgrad_multi_work_floats(FEN_WGRAD_MAXJOBS + 1, a.data()) == 0);
    const size_t one = fen_wgrad_work_floats(&a[0]);
    EXPECT(one == (size_t)256 * (64 * 64 * 9 + 64));
    EXPECT(fen_wgrad_multi_work_floats(4, a.data()) == one);
    for (int n : {1, 7, FEN_WGRAD_MAXJOBS}) EXPECT(fen_wgrad_multi_work_floats(n, a.data()) > 0);
    a[2].H = 32;
    EXPECT(fen_wgrad3x3_multi(4, a.data(), nullptr) == FEN_EINVAL);
    a[2].H = 64, a[3].x = nullptr;
    EXPECT(fen_wgrad3x3_multi(4, a.data(), nullptr) == FEN_EINVAL);
}

static void pack_tables() {
    // the post-step re-pack table of a full 6x10 network's 131 convs + the upsampler / tail
    const int nj = 140;
    std::vector<fen_pack_job> jobs(nj);
    for (int i = 0; i < nj; ++i)
        jobs[i] = fen_pack_job{(const float*)fake(2 * i), fake(2 * i + 1), i % 3, i % 3 == 1 ? 256 : 64, 64};
    std::vector<char> tab(fen_pack_table_bytes(nj));
    size_t total = 0;
    EXPECT(fen_pack_table(FEN_BF16, nj, jobs.data(), tab.data(), &total) == FEN_OK && total > 0);
    EXPECT(fen_pack_table(FEN_BF16, 0, jobs.data(), tab.data(), &total) == FEN_EINVAL);
    jobs[5].mode = 3;
    EXPECT(fen_pack_table(FEN_BF16, nj, jobs.data(), tab.data(), &total) == FEN_EINVAL);
    EXPECT(fen_pack_multi(FEN_BF16, 0, nullptr, 0, nullptr) == FEN_EINVAL);
}

static void chain_tables() {
    const int B = 2, H = 64, nb = 10, G = 6;
    const size_t nbytes = fen_group_strip_chain_work_bytes(B, H, G);
    EXPECT(nbytes > fen_group_strip_work_bytes(B, H));
    EXPECT(fen_group_strip_chain_work_bytes(B, 12, G) == 0);
    std::vector<fen_group_strip_desc> ds(G);
    for (int g = 0; g < G; ++g) {
        fen_group_strip_desc& d = ds[g];
        std::memset(&d, 0, sizeof d);
        d.dtype = FEN_BF16, d.B = B, d.H = H, d.W = 64, d.C = 64, d.Cr = 16, d.nb = nb, d.res_scale = 0.2f;
        d.x = fake(g + 1), d.y = fake(g + 2);
        for (int j = 0; j < nb; ++j) {
            d.w1[j] = d.w2[j] = fake(100 + j);
            d.b1[j] = d.b2[j] = d.alpha[j] = d.fc1[j] = d.fc2[j] = (const float*)fake(200 + j);
        }
        d.wg = fake(300), d.bg = (const float*)fake(301);
        d.work = fake(400), d.work_bytes = nbytes;
    }
    ds[1].x = fake(90);                                                  // not a chain
    EXPECT(fen_group_strip_chain(ds.data(), G, nullptr, nullptr) == FEN_EINVAL);
    EXPECT(fen_group_strip_chain_prepare(ds.data(), G, nullptr, nullptr) == FEN_EINVAL);
    ds[1].x = ds[0].y;
    fen_group_strip_chain_tail t{fake(500), (const float*)fake(501), ds[0].x, ds[G - 1].y};
    EXPECT(fen_group_strip_chain_prepare(ds.data(), G, &t, nullptr) == FEN_EINVAL);   // tail writes the body's output
    t.y = fake(600);
    // a valid chain: the table is built and hashed on the host; without a GPU the copy-kernel
    // launch then fails (FEN_EHIP) -- ASan covers everything before it
    const int rc = fen_group_strip_chain_prepare(ds.data(), G, &t, nullptr);
    EXPECT(rc == FEN_OK || rc == FEN_EHIP);
    std::vector<fen_group_strip_desc> big(13, ds[0]);
    for (int g = 0; g < 13; ++g) big[g].nb = 19, big[g].x = fake(g + 1), big[g].y = fake(g + 2);
    EXPECT(fen_group_strip_chain_prepare(big.data(), 13, nullptr, nullptr) == FEN_EUNSUPPORTED);
}

static void status_and_rccl() {
    EXPECT(std::strncmp(fen_status_string(FEN_ERCCL), "FEN_ERCCL", 9) == 0);
    EXPECT(fen_rccl_allreduce_bucket(nullptr, nullptr, 16, nullptr) == FEN_EINVAL);
    EXPECT(fen_rccl_init(nullptr, nullptr, 1, 0, 0) == FEN_EINVAL);
    void* h = nullptr;
    unsigned char uid[128] = {0};
    EXPECT(fen_rccl_init(&h, uid, 2, 2, 0) == FEN_EINVAL);
    EXPECT(fen_rccl_check(nullptr) == FEN_EINVAL);
    EXPECT(fen_rccl_destroy(nullptr) == FEN_OK);
    EXPECT(fen_rccl_library() != nullptr);                               // dlopen / dlsym path
    EXPECT(fen_last_rccl_error() != nullptr);
    int* w = (int*)std::malloc(sizeof(int));
    *w = 3;
    EXPECT(fen_status_take(w) == 3 && *w == 0);
    EXPECT(fen_status_take(w) == 0);
    EXPECT(fen_status_take(nullptr) == 0);
    std::free(w);
}

static void misc_refusals() {
    EXPECT(fen_rcab_deferred(nullptr, nullptr) == FEN_EINVAL);
    EXPECT(fen_group_strip(nullptr, nullptr) == FEN_EINVAL);
    EXPECT(fen_group_strip_bwd(nullptr, nullptr) == FEN_EINVAL);
    EXPECT(fen_rcab_c128(nullptr, nullptr) == FEN_EINVAL);
    EXPECT(fen_rcab_bwd(nullptr, nullptr) == FEN_EINVAL);
    EXPECT(fen_colsum_multi(0, nullptr, nullptr) == FEN_EINVAL);
    EXPECT(fen_ssim_ex(FEN_BF16, 2, 3, 64, 64, nullptr, nullptr, nullptr, 11, 1e-4f, 9e-4f, nullptr, nullptr, 1.f, 2,
                       (float*)fake(0), nullptr) == FEN_EINVAL);
    EXPECT(fen_bicubic_down4(0, 3, 256, 256, nullptr, nullptr, nullptr) == FEN_EINVAL);
}

// `asan_check overflow`: hands fen_pack_table a table one job too short -- the library's own
// write past it must be caught (proves the host half of libfen_hip_asan.so is instrumented)
static int overflow_selftest() {
    const int nj = 8;
    std::vector<fen_pack_job> jobs(nj, fen_pack_job{(const float*)fake(0), fake(1), 0, 64, 64});
    char* tab = (char*)std::malloc(fen_pack_table_bytes(nj - 1));
    size_t total = 0;
    const int rc = fen_pack_table(FEN_BF16, nj, jobs.data(), tab, &total);
    std::free(tab);
    std::printf("overflow self-test NOT caught (rc %d)\n", rc);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::strcmp(argv[1], "overflow") == 0) return overflow_selftest();
    pure_queries();
    conv_refusals();
    wgrad_tables();
    pack_tables();
    chain_tables();
    status_and_rccl();
    misc_refusals();
    if (g_fail) {
        std::fprintf(stderr, "asan_check: %d expectation(s) failed\n", g_fail);
        return 1;
    }
    std::printf("asan_check: all host paths clean under AddressSanitizer\n");
    return 0;
}
