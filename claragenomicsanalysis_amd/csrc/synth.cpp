// Synthetic ONT-like inputs for bench.py and the parity tests: a restatement of
// the reference's generators (common/base/include/claraparabricks/genomeworks/
// utils/genomeutils.hpp:26-126) on std::minstd_rand and the standard library's
// distributions, so that window w of a config is exactly the reference's
// generate_random_sequences(generate_random_genome(L, rng(seed)), ...) output.
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace
{
const char kAlphabet[4] = {'A', 'C', 'G', 'T'};

std::string random_genome(int32_t length, std::minstd_rand& rng)
{
    std::uniform_int_distribution<int32_t> pick(0, 3);
    std::string g;
    g.reserve(size_t(length));
    for (int32_t i = 0; i < length; i++)
        g += kAlphabet[pick(rng)];
    return g;
}

// generate_random_sequence over the full backbone range (genomeutils.hpp:38-105)
std::string mutate(const std::string& backbone, std::minstd_rand& rng, int max_mut, int max_ins, int max_del)
{
    std::uniform_int_distribution<int> base(0, 3);
    std::uniform_real_distribution<double> coin(0, 1);
    const int range = int(backbone.size());
    std::string s   = backbone;
    for (int j = 0; j < std::min(max_del, range); j++)
    {
        if (coin(rng) > 0.5)
        {
            std::uniform_int_distribution<int> at(0, int(s.size()) - 1);
            s.erase(size_t(at(rng)), 1);
        }
    }
    for (int j = 0; j < std::min(max_ins, range); j++)
    {
        if (coin(rng) > 0.5)
        {
            std::uniform_int_distribution<int> at(0, int(s.size()));
            int p = at(rng);
            int b = base(rng);
            s.insert(size_t(p), 1, kAlphabet[b]);
        }
    }
    if (!s.empty())
    {
        std::uniform_int_distribution<int> at(0, int(s.size()) - 1);
        for (int j = 0; j < std::min(max_mut, range); j++)
        {
            if (coin(rng) > 0.5)
            {
                int p = at(rng);
                int b = base(rng);
                s[size_t(p)] = kAlphabet[b];
            }
        }
    }
    return s;
}
} // namespace

extern "C" {

// Windows w = 0..n-1: rng = minstd_rand(first_seed + w); backbone of
// backbone_len bases; reads = backbone + (num_reads-1) mutated copies
// (generate_random_sequences, genomeutils.hpp:107-120).  Bases are packed into
// bases_out (capacity bases_cap), read lengths into lens_out
// (n * num_reads).  Returns total bases, or -1 if bases_cap is too small.
int64_t gwamd_synth_poa_windows(int32_t first_seed, int32_t n, int32_t backbone_len, int32_t num_reads,
                                int32_t max_mut, int32_t max_ins, int32_t max_del, uint8_t* bases_out,
                                int64_t bases_cap, int32_t* lens_out)
{
    // windows are independent (one generator per window): chunks of windows
    // are generated on host threads, then packed in window order
    const int32_t chunk = 512;
    const int32_t nchunks = (n + chunk - 1) / chunk;
    std::vector<std::string> text(size_t(std::max(nchunks, 0)));
    auto gen = [&](int32_t c) {
        std::string& out = text[size_t(c)];
        for (int32_t w = c * chunk; w < std::min(n, (c + 1) * chunk); w++)
        {
            std::minstd_rand rng(uint32_t(first_seed + w));
            const std::string bb = random_genome(backbone_len, rng);
            for (int32_t r = 0; r < num_reads; r++)
            {
                const std::string s = (r == 0) ? bb : mutate(bb, rng, max_mut, max_ins, max_del);
                out += s;
                lens_out[size_t(w) * num_reads + r] = int32_t(s.size());
            }
        }
    };
    const int32_t nth = std::max(1, std::min<int32_t>(nchunks, int32_t(std::min(16u, std::thread::hardware_concurrency()))));
    std::vector<std::thread> th;
    for (int32_t t = 0; t < nth; t++)
        th.emplace_back([&, t] {
            for (int32_t c = t; c < nchunks; c += nth)
                gen(c);
        });
    for (auto& t : th)
        t.join();
    int64_t off = 0;
    for (const auto& s : text)
    {
        if (off + int64_t(s.size()) > bases_cap)
            return -1;
        std::memcpy(bases_out + off, s.data(), s.size());
        off += int64_t(s.size());
    }
    return off;
}

// Pairs i = 0..n-1 (cudaaligner/benchmarks/main.cpp:109-115 recipe):
// rng = minstd_rand(first_seed + i); target = random genome of target_len;
// query = mutate(target) truncated to query_cap.  Query/target are written at
// stride `stride` into q_out / t_out.
int32_t gwamd_synth_pairs(int32_t first_seed, int32_t n, int32_t target_len, int32_t query_cap, int32_t max_mut,
                          int32_t max_ins, int32_t max_del, uint8_t* q_out, uint8_t* t_out, int32_t stride,
                          int32_t* q_len, int32_t* t_len)
{
    for (int32_t i = 0; i < n; i++)
    {
        std::minstd_rand rng(uint32_t(first_seed + i));
        const std::string t = random_genome(target_len, rng);
        std::string q        = mutate(t, rng, max_mut, max_ins, max_del);
        if (int32_t(q.size()) > query_cap)
            q.resize(size_t(query_cap));
        if (int32_t(t.size()) > stride || int32_t(q.size()) > stride)
            return -1;
        std::memcpy(t_out + size_t(i) * stride, t.data(), t.size());
        std::memcpy(q_out + size_t(i) * stride, q.data(), q.size());
        t_len[i] = int32_t(t.size());
        q_len[i] = int32_t(q.size());
    }
    return 0;
}

} // extern "C"
