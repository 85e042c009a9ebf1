// rs_dropin.cpp -- exercises include/ezpwd_amd/rs (the ezpwd::RS<N,K> call surface) through the
// overloads ezpwd users call: string / vector / array / pair / pointer encode, and decode with
// erasure + position vectors (rs_base:210-408, 868-904, 1130-1242).  It prints one record per
// trial; tests/test_cpp_dropin.py checks every record against the oracle.
//
// Usage: rs_dropin [trials]   -> exit 0; prints "NODEV <msg>" and exits 3 when no GPU is usable.
#define EZPWD_AMD_AS_EZPWD
#include <ezpwd_amd/rs>

#include <cstdio>
#include <cstdlib>
#include <iostream>

static uint64_t s_state = 0x5EED0D0Bull;
static uint64_t next() {   // splitmix64
    uint64_t z = (s_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <typename V> static void hex(const char *tag, const V &v) {
    std::printf(" %s=", tag);
    for (auto x : v) std::printf("%x,", unsigned(x));
}

static int failures = 0;
#define CHECK(c)                                                                \
    do {                                                                        \
        if (!(c)) {                                                             \
            std::printf("CHECK FAILED line %d: %s\n", __LINE__, #c);            \
            ++failures;                                                         \
        }                                                                       \
    } while (0)

// One trial: encode `len` random symbols with every overload, corrupt, decode, print.
template <class RS, typename T>
static void trial(const char *name, const RS &rs, unsigned len, unsigned nerr, unsigned neras) {
    const unsigned NR = rs.nroots(), msk = (1u << rs.symbol()) - 1;
    std::vector<T> data(len);
    for (auto &x : data) x = T(next() & msk);

    // vector (parity appended), vector + separate parity, pointer form, pair form
    std::vector<T> cw = data;
    CHECK(rs.encode(cw) == int(NR));
    std::vector<T> par;
    CHECK(rs.encode(data, par) == int(NR));
    std::vector<T> par2(NR);
    CHECK(rs.encode(data.data(), len, par2.data()) == int(NR));
    std::vector<T> cw3 = data;
    cw3.resize(len + NR);
    CHECK(rs.encode(std::make_pair(cw3.data(), cw3.data() + cw3.size())) == int(NR));
    CHECK(std::equal(par.begin(), par.end(), cw.begin() + len));
    CHECK(par == par2);
    CHECK(cw3 == cw);

    // corrupt nerr + neras distinct positions; the last neras of them are signalled as erasures
    std::vector<T> bad = cw;
    std::vector<unsigned> where;
    while (where.size() < nerr + neras) {
        const unsigned p = unsigned(next() % (len + NR));
        if (std::find(where.begin(), where.end(), p) == where.end()) where.push_back(p);
    }
    for (unsigned p : where) bad[p] ^= T(1 + next() % msk);
    std::vector<unsigned> eras(where.end() - neras, where.end());
    std::vector<T> fixed = bad;
    std::vector<unsigned> pos;
    const int r = rs.decode(fixed, eras, &pos);
    std::printf("REC %s len=%u r=%d", name, len, r);
    hex("data", data);
    hex("parity", par);
    hex("bad", bad);
    hex("eras", eras);
    hex("pos", pos);
    hex("fixed", fixed);
    std::printf("\n");
    if (nerr * 2 + neras <= NR) {
        CHECK(r == int(nerr + neras));
        CHECK(fixed == cw);
        CHECK(ezpwd::strength<64>(r, eras, pos) >= -1);
    }
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? std::atoi(argv[1]) : 8;
    try {
        ezpwd::RS<255, 223> rs255;
        ezpwd::RS<31, 27> rs31;          // 5-bit symbols in uint8_t: the masked path
        ezpwd::RS<1023, 1007> rs1023;    // uint16_t symbols
        ezpwd::RS_CCSDS<255, 223> ccsds; // dual basis
        std::cout << "# " << rs255 << " " << rs31 << " " << rs1023 << " " << ccsds << "\n";
        for (int t = 0; t < trials; ++t) {
            trial<decltype(rs255), uint8_t>("RS255_223", rs255, 1 + unsigned(next() % 223), t % 9, t % 5);
            trial<decltype(rs31), uint8_t>("RS31_27", rs31, 1 + unsigned(next() % 27), t % 3, t % 2);
            trial<decltype(rs1023), uint16_t>("RS1023_1007", rs1023, 1 + unsigned(next() % 1007), t % 5, t % 4);
            trial<decltype(ccsds), uint8_t>("CCSDS255_223", ccsds, 1 + unsigned(next() % 223), t % 9, t % 5);
        }
        // string forms and the error behaviour of the reference (rs_base:875-877)
        std::string s = "The quick brown fox jumps over the lazy dog";
        const std::string orig = s;
        rs255.encode(s);
        CHECK(s.size() == orig.size() + 32);
        s[3] ^= 0x55;
        std::vector<unsigned> pos;
        CHECK(rs255.decode(s, std::vector<unsigned>(), &pos) == 1);
        CHECK(pos.size() == 1 && pos[0] == 3);
        CHECK(s.substr(0, orig.size()) == orig);
        bool threw = false;
        try {
            std::vector<uint8_t> big(224);
            std::vector<uint8_t> p;
            rs255.encode(big, p);
        } catch (const std::runtime_error &) {
            threw = true;
        }
        CHECK(threw);
    } catch (const std::runtime_error &e) {
        std::printf("NODEV %s\n", e.what());
        return 3;
    }
    std::printf("DONE failures=%d\n", failures);
    return failures ? 1 : 0;
}
