/* A plain C99 consumer of include/fheregex.h, built and run by
 * tests/test_host.py::test_c_abi_consumer (gcc, no GPU): the boundary is usable
 * from C exactly as declared (the Rust extern block of INTEGRATION.md binds the
 * same symbols).  Host-only context (device -1): reference parse / Err / panic
 * behaviour (parser.rs:146-351, engine.rs:189-190), the reference counters of
 * has_match on a golden vector (engine.rs:256-280), the client key loaded from the
 * fixture, and GPU entry points refusing loudly with FR_ERR_NO_DEVICE.
 * With a second argument "gpu" (tests/test_gpu.py::test_c_abi_consumer_gpu) it also
 * runs the engine end to end on device 0 from C: server key, device encryption of the
 * content (encrypt_str, ciphertext.rs:32-40), has_match (engine.rs:8-42), the
 * result downloaded and decrypted under the fixture key -- planted and absent.
 * Usage: c_abi_consumer <path to tests/golden/client_key> [gpu]; exit status 0 = pass. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fheregex.h"

static int failures = 0;
#define CHECK(cond, ...)                           \
    do {                                           \
        if (!(cond)) {                             \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);          \
            fprintf(stderr, "\n");                 \
            ++failures;                            \
        }                                          \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s client_key\n", argv[0]);
        return 2;
    }
    fr_params p;
    CHECK(fr_default_params(&p) == FR_OK, "default params");
    CHECK(p.k == 1 && p.N == 2048 && p.n == 742 && p.ks_base_log == 3 && p.ks_level == 5 && p.pbs_base_log == 23 &&
              p.pbs_level == 1,
          "PARAM_MESSAGE_2_CARRY_2: k=%d N=%d n=%d", p.k, p.N, p.n);

    /* parser: canonical AST, the reference's Err and panic */
    char ast[512];
    CHECK(fr_parse("/abc/", ast, sizeof ast) == FR_OK && strlen(ast) > 0, "parse /abc/");
    CHECK(fr_parse("/[a-z0-9]+/", ast, sizeof ast) == FR_ERR_PARSE, "[a-z0-9] is Err in the reference grammar");
    CHECK(strlen(fr_last_error()) > 0, "error message set");

    /* symbolic has_match with the reference's counters: /abc/ on "qqabcq" */
    fr_plain_result r;
    memset(&r, 0, sizeof r);
    CHECK(fr_plain_match("qqabcq", 6, "/abc/", 0, 6, FR_LOWER_FAITHFUL, &r) == FR_OK, "plain match");
    CHECK(r.result_recorded == 1 && r.result_lowered == 1, "/abc/ in qqabcq: %d %d", r.result_recorded,
          r.result_lowered);
    /* golden vectors with the reference's counters (tests/golden/engine_vectors.json) */
    memset(&r, 0, sizeof r);
    CHECK(fr_plain_match("ab", 2, "/ab/", 0, 2, FR_LOWER_FAITHFUL, &r) == FR_OK, "plain match ab");
    CHECK(r.result_recorded == 1 && r.ct_ops == 3 && r.cache_hits == 0, "/ab/ on ab: %d ops %llu hits %llu",
          r.result_recorded, (unsigned long long)r.ct_ops, (unsigned long long)r.cache_hits);
    memset(&r, 0, sizeof r);
    CHECK(fr_plain_match("ab", 2, "/a?b/", 0, 2, FR_LOWER_FAITHFUL, &r) == FR_OK, "plain match a?b");
    CHECK(r.result_recorded == 1 && r.ct_ops == 6 && r.cache_hits == 1, "/a?b/ on ab: %d ops %llu hits %llu",
          r.result_recorded, (unsigned long long)r.ct_ops, (unsigned long long)r.cache_hits);
    memset(&r, 0, sizeof r);
    CHECK(fr_plain_match("qqabxq", 6, "/abc/", 0, 6, FR_LOWER_THRESHOLD, &r) == FR_OK, "plain match (absent)");
    CHECK(r.result_recorded == 0 && r.result_lowered == 0, "/abc/ not in qqabxq");

    /* a host-only context: keys load, GPU entry points refuse */
    fr_ctx* ctx = NULL;
    CHECK(fr_ctx_create(&p, -1, &ctx) == FR_OK && ctx, "host-only context");
    FILE* f = fopen(argv[1], "rb");
    CHECK(f != NULL, "open %s", argv[1]);
    if (f && ctx) {
        fseek(f, 0, SEEK_END);
        const long len = ftell(f);
        fseek(f, 0, SEEK_SET);
        unsigned char* blob = (unsigned char*)malloc((size_t)len);
        CHECK(blob && fread(blob, 1, (size_t)len, f) == (size_t)len, "read client key");
        CHECK(fr_load_client_key(ctx, blob, (size_t)len) == FR_OK, "load client key: %s", fr_last_error());
        /* the writer gives the fixture back byte for byte (engine.rs:238-246) */
        size_t need = 0;
        CHECK(fr_serialize_client_key(ctx, NULL, 0, &need) == FR_OK && need == (size_t)len, "client key size %zu",
              need);
        unsigned char* back = (unsigned char*)malloc(need ? need : 1);
        CHECK(back && fr_serialize_client_key(ctx, back, need, &need) == FR_OK && memcmp(back, blob, need) == 0,
              "serialize(load(fixture)) == fixture");
        /* a fresh key (gen_keys_radix, ciphertext.rs:44) round-trips through the loader */
        fr_ctx* gen = NULL;
        CHECK(fr_ctx_create(&p, -1, &gen) == FR_OK && gen, "second host context");
        if (gen && back) {
            CHECK(fr_gen_client_key(gen, 7) == FR_OK, "gen client key: %s", fr_last_error());
            CHECK(fr_serialize_client_key(gen, back, need, &need) == FR_OK && need == (size_t)len, "generated size");
            CHECK(fr_load_client_key(gen, back, need) == FR_OK, "load generated key: %s", fr_last_error());
            fr_ctx_destroy(gen);
        }
        free(back);
        free(blob);
        /* a server holding only the exported server key (has_match(sk, ..), engine.rs:8) */
        size_t kl = 0, bl = 0;
        CHECK(fr_gen_server_key(ctx, 42) == FR_OK, "host server key: %s", fr_last_error());
        CHECK(fr_server_key_sizes(ctx, &kl, &bl) == FR_OK && kl && bl, "server key sizes");
        uint64_t* ksk = (uint64_t*)malloc(8 * kl);
        uint64_t* bsk = (uint64_t*)malloc(8 * bl);
        uint64_t* bsk2 = (uint64_t*)malloc(8 * bl);
        fr_ctx* srv = NULL;
        CHECK(fr_ctx_create(&p, -1, &srv) == FR_OK && srv, "server context");
        if (ksk && bsk && bsk2 && srv) {
            CHECK(fr_export_server_key(ctx, ksk, kl, bsk, bl) == FR_OK, "export: %s", fr_last_error());
            CHECK(fr_load_server_key(srv, ksk, kl, bsk, bl - 1) == FR_ERR_INVALID, "short bsk refused");
            CHECK(fr_load_server_key(srv, ksk, kl, bsk, bl) == FR_OK, "load server key: %s", fr_last_error());
            CHECK(fr_export_server_key(srv, NULL, 0, bsk2, bl) == FR_OK && memcmp(bsk, bsk2, 8 * bl) == 0,
                  "export(load(k)) == k");
            CHECK(fr_serialize_client_key(srv, NULL, 0, &need) == FR_ERR_NO_KEY, "the server has no client key");
        }
        if (srv) fr_ctx_destroy(srv);
        free(ksk);
        free(bsk);
        free(bsk2);
        fr_ct content[1] = {0};
        fr_ct out = 0;
        CHECK(fr_has_match(ctx, content, 1, "/a/", &out, NULL) == FR_ERR_NO_DEVICE, "has_match needs a device");
    }
    if (f) fclose(f);
    if (ctx) CHECK(fr_ctx_destroy(ctx) == FR_OK, "destroy");

    if (argc > 2 && strcmp(argv[2], "gpu") == 0) {
        /* the engine end to end on device 0 */
        fr_ctx* g = NULL;
        CHECK(fr_ctx_create(&p, 0, &g) == FR_OK && g, "device context: %s", fr_last_error());
        f = fopen(argv[1], "rb");
        if (g && f) {
            fseek(f, 0, SEEK_END);
            const long len = ftell(f);
            fseek(f, 0, SEEK_SET);
            unsigned char* blob = (unsigned char*)malloc((size_t)len);
            CHECK(blob && fread(blob, 1, (size_t)len, f) == (size_t)len, "read client key");
            CHECK(fr_load_client_key(g, blob, (size_t)len) == FR_OK, "load client key: %s", fr_last_error());
            free(blob);
            CHECK(fr_gen_server_key(g, 42) == FR_OK, "server key: %s", fr_last_error());
            const char* texts[2] = {"the quick abc fox", "the quick abx fox"};
            const uint64_t expect[2] = {1, 0};
            const size_t lwe = (size_t)p.k * (size_t)p.N + 1;
            uint64_t* blocks = (uint64_t*)malloc(4 * lwe * sizeof(uint64_t));
            for (int t = 0; t < 2; ++t) {
                const size_t n = strlen(texts[t]);
                fr_ct chars[32];
                CHECK(fr_encrypt_upload_str(g, texts[t], n, 7 + (uint64_t)t, chars) == FR_OK, "encrypt: %s",
                      fr_last_error());
                fr_ct res = 0;
                fr_match_stats st;
                memset(&st, 0, sizeof st);
                CHECK(fr_has_match(g, chars, n, "/abc/", &res, &st) == FR_OK, "has_match: %s", fr_last_error());
                CHECK(fr_download_radix(g, res, blocks) == FR_OK, "download: %s", fr_last_error());
                uint64_t v = 99;
                CHECK(fr_decrypt_radix(g, blocks, &v) == FR_OK && v == expect[t], "/abc/ on '%s': %llu",
                      texts[t], (unsigned long long)v);
                CHECK(st.blind_rotations > 0 && st.levels > 0, "stats filled");
                fr_release(g, res);
                for (size_t q = 0; q < n; ++q) fr_release(g, chars[q]);
            }
            fr_ct one[1];
            CHECK(fr_encrypt_upload_str(g, "a", 1, 9, one) == FR_OK, "encrypt one char");
            fr_ct bad = 0;
            CHECK(fr_has_match(g, one, 1, "/[a-z0-9]+/", &bad, NULL) == FR_ERR_PARSE,
                  "the reference's Err on the device path");
            fr_release(g, one[0]);
            free(blocks);
        }
        if (f) fclose(f);
        if (g) CHECK(fr_ctx_destroy(g) == FR_OK, "destroy device context");
    }

    if (failures) {
        fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    printf("c_abi_consumer: ok\n");
    return 0;
}
