// verifier <base>: src/bin/verifier.rs:9-25. Prints `true` or `false`.
#include <stdio.h>

#include <fstream>
#include <sstream>
#include <string>

#include "bpg.h"

static bool slurp(const std::string &path, std::string &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "missing argument\n"); return 1; }
    std::string base = argv[1], inst, coms, proof, gadgets;
    if (!slurp(base + ".inst", inst) || !slurp(base + ".coms", coms) || !slurp(base + ".proof", proof) ||
        !slurp(base + ".gadgets", gadgets)) {
        fprintf(stderr, "unable to read files\n");
        return 1;
    }
    bool ok = c_verify(base.c_str(), inst.c_str(), gadgets.c_str(), coms.c_str(), (const uint8_t *)proof.data(),
                       proof.size());
    if (!ok && bpg_last_error()[0]) fprintf(stderr, "%s\n", bpg_last_error());
    printf("%s\n", ok ? "true" : "false");
    return 0;
}
