// Fuzz: the AVX2 de-stuffer against the scalar one (random bytes rich in
// 0xFF, stuffing, RSTn and end markers).  Built and run by tests/test_jpeg_host.py.
#include "../../wicca_amd/csrc/jpeg_host.cpp"
#include <cstdio>
#include <random>
int main() {
    std::mt19937 rng(1);
    int bad = 0;
    for (int t = 0; t < 20000; ++t) {
        size_t n = rng() % 300 + 1;
        std::vector<uint8_t> in(n);
        for (auto& b : in) {
            uint32_t r = rng() % 16;
            b = r < 3 ? 0xFF : r == 3 ? 0x00 : r == 4 ? (uint8_t)(0xD0 + rng() % 8) : r == 5 ? 0xD9 : (uint8_t)rng();
        }
        std::vector<uint8_t> o1(n + 64, 0xAA), o2(n + 64, 0xAA);
        std::vector<int64_t> s1, s2;
        s1.assign(1, 0); s2.assign(1, 0);
        bool r1 = false, r2 = false;
        size_t a = wicca::destuff_scalar(in.data(), n, 0, o1.data(), 0, s1, r1);
        size_t b = wicca::destuff_avx2(in.data(), n, o2.data(), s2, r2);
        if (a != b || s1 != s2 || r1 != r2 || memcmp(o1.data(), o2.data(), a) != 0) { if (bad++ < 5) printf("mismatch t=%d n=%zu a=%zu b=%zu\n", t, n, a, b); }
    }
    printf("bad=%d\n", bad);
    return bad != 0;
}
