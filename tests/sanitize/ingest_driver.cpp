// Sanitizer driver for the native VCF ingest (2dsfs-scan_amd/csrc/vcf_ingest.cpp, include/sfs2d_ingest.h):
// built with -fsanitize=address,undefined (or thread) together with the parser's source, it reads
// each (vcf, popmap) given on the command line with several thread counts, touches every output
// column and prints one digest line per read, which tests/test_sanitize.py compares with the normal
// library's results.  Test infrastructure only.
//   usage: ingest_driver <threads,threads,...> <vcf> <popmap> [<vcf> <popmap> ...]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sfs2d_ingest.h"

int main(int argc, char** argv) {
  if (argc < 4 || (argc - 2) % 2) {
    std::fprintf(stderr, "usage: %s threads vcf popmap [vcf popmap ...]\n", argv[0]);
    return 2;
  }
  std::vector<int> threads;
  for (char* t = std::strtok(argv[1], ","); t; t = std::strtok(nullptr, ",")) threads.push_back(std::atoi(t));
  for (int a = 2; a + 1 < argc; a += 2) {
    for (int nt : threads) {
      sfs2d_vcf* v = nullptr;
      const int rc = sfs2d_vcf_read(argv[a], argv[a + 1], nt, &v);
      if (rc != 0) {
        std::printf("%s threads=%d rc=%d err=%s\n", argv[a], nt, rc, sfs2d_vcf_last_error());
        continue;
      }
      const int64_t n = sfs2d_vcf_num_records(v);
      const int32_t np = sfs2d_vcf_num_pops(v), nc = sfs2d_vcf_num_chroms(v), na = sfs2d_vcf_num_annotations(v);
      const int32_t *chrom = nullptr, *ann = nullptr, *calls = nullptr;
      const int64_t *pos = nullptr, *pos_off = nullptr;
      const char* blob = nullptr;
      const uint8_t* alleles = nullptr;
      sfs2d_vcf_columns(v, &chrom, &pos, &blob, &pos_off, &ann, &alleles, &calls);
      uint64_t h = 1469598103934665603ull;   // FNV-1a over every column
      auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
      for (int64_t i = 0; i < n; ++i) {
        mix((uint64_t)chrom[i]); mix((uint64_t)pos[i]); mix((uint64_t)ann[i]);
        mix(alleles[2 * i]); mix(alleles[2 * i + 1]);
        for (int64_t b = pos_off[i]; b < pos_off[i + 1]; ++b) mix((uint8_t)blob[b]);
        for (int32_t p = 0; p < np; ++p) { mix((uint64_t)(int64_t)calls[(i * np + p) * 2]); mix((uint64_t)(int64_t)calls[(i * np + p) * 2 + 1]); }
      }
      std::string names;
      for (int32_t c = 0; c < nc; ++c) names += std::string(sfs2d_vcf_chrom_name(v, c)) + ",";
      for (int32_t p = 0; p < np; ++p) names += std::string(sfs2d_vcf_pop_name(v, p)) + ";";
      for (int32_t k = 0; k < na; ++k) names += std::string(sfs2d_vcf_annotation(v, k)) + "|";
      for (char ch : names) mix((uint8_t)ch);
      std::printf("%s threads=%d records=%lld pops=%d chroms=%d anns=%d digest=%016llx\n", argv[a], nt, (long long)n,
                  np, nc, na, (unsigned long long)h);
      sfs2d_vcf_free(v);
    }
  }
  return 0;
}
