// prover <base> [--seed S]: src/bin/prover.rs:16-30. Reads <base>.inst,
// <base>.wtns, <base>.gadgets; writes <base>.coms and <base>.proof. The
// transcript label is the base path string, as in the reference (:17).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
    std::string base = argv[1];
    for (int i = 2; i + 1 < argc; i++)
        if (!strcmp(argv[i], "--seed")) bpg_set_seed(strtoull(argv[i + 1], nullptr, 0));
    std::string inst, wtns, gadgets;
    if (!slurp(base + ".inst", inst) || !slurp(base + ".wtns", wtns) || !slurp(base + ".gadgets", gadgets)) {
        fprintf(stderr, "unable to read instance file\n");
        return 1;
    }
    struct ProofArtifacts *a = c_prove(base.c_str(), inst.c_str(), wtns.c_str(), gadgets.c_str());
    if (!a) { fprintf(stderr, "unable to generate proof from provided files: %s\n", bpg_last_error()); return 1; }
    printf("%llu\n", (unsigned long long)bpg_last_num_constraints());
    std::ofstream(base + ".coms", std::ios::binary) << a->commitments;
    std::ofstream(base + ".proof", std::ios::binary).write((const char *)a->proof, (std::streamsize)a->proof_len);
    free_proof(a);
    return 0;
}
