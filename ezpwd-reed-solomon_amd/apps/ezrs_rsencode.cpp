// ezrs_rsencode -- the rsencode streaming codec (rsencode.C) on the MI355X engine.
//
//   ezrs_rsencode [-e|--encode] [-d|--decode] [-c|--chunk N] [-n|--codeword N] [-p|--parity P]
//                 [<input> [<output>]]
//
// Same wire format and failure behaviour as the reference's rsencode (rsencode.C:52-163): chunks
// of N data symbols each followed by P parity symbols of RS(codeword, codeword - parity), symbols
// wider than 8 bits big-endian; decode corrects and strips the parity, passing a chunk it cannot
// correct on as the decoder left it.  Where the reference fixes the codec at compile time
// (RSCODEWORD / RSPARITY) this tool takes it on the command line (defaults: RS(255,223), 128-symbol
// chunks, as rsencode).  Input and output default to stdin / stdout ("-").  The file is processed in
// blocks of many chunks, each block one batch on the GPU (include/ezrs.h ezrs_stream_*).
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ezrs.h"

namespace {

size_t read_full(FILE *f, unsigned char *buf, size_t n) {
    size_t got = 0;
    while (got < n) {
        const size_t r = std::fread(buf + got, 1, n - got, f);
        if (r == 0) break;
        got += r;
    }
    return got;
}

int usage(const char *msg) {
    std::fprintf(stderr, "%s\n"
                 "    -e|--encode   -- R-S encode, adding parity (default)\n"
                 "    -d|--decode   -- R-S decode, correcting errors and removing parity\n"
                 "    -c|--chunk    -- data symbols per chunk; default: 128\n"
                 "    -n|--codeword -- R-S codeword size 2^m-1; default: 255\n"
                 "    -p|--parity   -- parity symbols; default: 32\n", msg);
    return 1;
}

} // namespace

int main(int argc, char **argv) {
    bool encoding = true;
    long chunk = 128, codeword = 255, parity = 32;
    std::vector<const char *> files;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto value = [&](long &dst) -> bool {
            if (i + 1 >= argc) return false;
            char *end = nullptr;
            dst = std::strtol(argv[++i], &end, 10);
            return end && *end == '\0' && dst > 0;
        };
        if (a == "-e" || a == "--encode") encoding = true;
        else if (a == "-d" || a == "--decode") encoding = false;
        else if (a == "-c" || a == "--chunk") { if (!value(chunk)) return usage("bad chunk size"); }
        else if (a == "-n" || a == "--codeword") { if (!value(codeword)) return usage("bad codeword size"); }
        else if (a == "-p" || a == "--parity") { if (!value(parity)) return usage("bad parity"); }
        else if (a.size() > 1 && a[0] == '-') return usage(("Invalid option: " + a).c_str());
        else files.push_back(argv[i]);
    }
    if (parity >= codeword) return usage("parity must be below the codeword size");
    ezrs_codec *rs = nullptr;
    int rc = ezrs_create_rs(&rs, (unsigned)codeword, (unsigned)(codeword - parity), 0);
    if (rc) {
        std::fprintf(stderr, "Error: cannot create RS(%ld,%ld) on the GPU: %s\n", codeword,
                     codeword - parity, ezrs_last_error());
        return 1;
    }
    ezrs_info info;
    ezrs_get_info(rs, &info);
    if ((unsigned long)chunk > info.load) {
        std::fprintf(stderr, "Error: chunk of %ld symbols exceeds RS(%ld,%ld) capacity\n", chunk,
                     codeword, codeword - parity);
        return 1;
    }
    FILE *in = stdin, *out = stdout;
    if (files.size() > 0 && std::strcmp(files[0], "-")) in = std::fopen(files[0], "rb");
    if (files.size() > 1 && std::strcmp(files[1], "-")) out = std::fopen(files[1], "wb");
    if (!in || !out) {
        std::fprintf(stderr, "Error: cannot open %s\n", !in ? files[0] : files[1]);
        return 1;
    }
    const size_t w = info.datum_bytes;
    const size_t per_chunk = encoding ? chunk * w : (chunk + info.nroots) * w;
    const size_t block = per_chunk * (size_t)(1u << 16);   // 64k chunks per GPU batch
    std::vector<unsigned char> ib(block), ob;
    size_t total = 0, failed = 0;
    int status = 0;
    for (;;) {
        const size_t got = read_full(in, ib.data(), block);
        total += got;
        if (got == 0) break;
        size_t n = 0, nf = 0;
        if (encoding) {
            ob.resize(ezrs_stream_encoded_bound(rs, got, (unsigned)chunk));
            rc = ezrs_stream_encode(rs, ib.data(), got, (unsigned)chunk, ob.data(), ob.size(), &n);
        } else {
            ob.resize(got);
            rc = ezrs_stream_decode(rs, ib.data(), got, (unsigned)chunk, ob.data(), ob.size(), &n, &nf);
        }
        failed += nf;
        if (n) std::fwrite(ob.data(), 1, n, out);
        if (rc == -EMSGSIZE) {                      // rsencode.C:110-111, 140-141
            std::fflush(out);
            std::fprintf(stderr, "Error after %zu bytes: Insufficient data for an RS(%ld,%ld) encoded chunk\n",
                         total, codeword, codeword - parity);
            status = 1;
            break;
        }
        if (rc) {
            std::fflush(out);
            std::fprintf(stderr, "Error after %zu bytes: %s (%d)\n", total, ezrs_last_error(), rc);
            status = 1;
            break;
        }
        if (got < block) break;
    }
    std::fflush(out);
    if (!encoding && failed && std::getenv("EZRS_RSENCODE_VERBOSE"))
        std::fprintf(stderr, "%zu chunk(s) could not be corrected\n", failed);
    if (in != stdin) std::fclose(in);
    if (out != stdout) std::fclose(out);
    ezrs_destroy(rs);
    return status;
}
