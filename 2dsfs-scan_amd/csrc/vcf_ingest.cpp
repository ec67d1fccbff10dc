// vcf_ingest.cpp -- multithreaded VCF(.gz / BGZF) + popmap parser behind include/sfs2d_ingest.h.
//
// Restates make_data_dict_vcf (uricchio/2DSFS-scan scripts/src/twoDSFS_class.py:36-138) for
// files of 1e7+ records: the reference spends ~15 us per SNP in Python string handling, which
// dominates end-to-end time once the scan itself runs on the GPU.
//
// Pipeline (all stages parallel where the format allows):
//   1. read the file; gzip members are located (BGZF: from the BSIZE extra field, so every block
//      is inflated independently into its slot of the text buffer; other gzip: one sequential
//      inflate over all members; no gzip magic: plain text);
//   2. the header block ('#' lines at the top) is read sequentially: popmap lookups build poplist;
//   3. the body is cut into line-aligned chunks, one per thread; each thread applies the
//      reference's per-line rules and keeps the records that reach the dict assignment (134);
//      a '#CHROM' line inside the body (poplist changes mid-file) reruns the body sequentially;
//   4. merge with dict semantics in file order: a key keeps its first slot, later records
//      overwrite its values.
// Errors stop at the first offending line in file order, as the reference's exception would.
#include <sched.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "sfs2d_ingest.h"

namespace {

thread_local std::string g_err;

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

struct Fail {
  int code;
  std::string msg;
};

bool read_file(const char* path, std::vector<unsigned char>& out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize(n > 0 ? (size_t)n : 0);
  const size_t got = n > 0 ? std::fread(out.data(), 1, (size_t)n, f) : 0;
  std::fclose(f);
  return got == out.size();
}

// ------------------------------------------------------------------------------------- inflate

struct Member {   // one BGZF block
  size_t off, cdata, clen;   // block start, deflate data offset / length
  uint32_t isize;
  size_t out;                // offset in the text buffer
};

// BGZF block list, or false when some member is not a BGZF block (then inflate sequentially)
bool bgzf_members(const std::vector<unsigned char>& z, std::vector<Member>& m) {
  size_t off = 0, out = 0;
  while (off < z.size()) {
    if (z.size() - off < 18 || z[off] != 0x1f || z[off + 1] != 0x8b || z[off + 2] != 8 || z[off + 3] != 4) return false;
    const size_t xlen = z[off + 10] | (z[off + 11] << 8);
    size_t p = off + 12, e = p + xlen, bsize = 0;
    if (e > z.size()) return false;
    while (p + 4 <= e) {
      const size_t sl = z[p + 2] | (z[p + 3] << 8);
      if (z[p] == 'B' && z[p + 1] == 'C' && sl == 2 && p + 6 <= e) bsize = (size_t)(z[p + 4] | (z[p + 5] << 8)) + 1;
      p += 4 + sl;
    }
    if (!bsize || off + bsize > z.size() || bsize < 12 + xlen + 8) return false;
    Member b;
    b.off = off;
    b.cdata = off + 12 + xlen;
    b.clen = bsize - 12 - xlen - 8;
    const unsigned char* t = &z[off + bsize - 4];
    b.isize = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
    b.out = out;
    out += b.isize;
    m.push_back(b);
    off += bsize;
  }
  return true;
}

bool inflate_raw(const unsigned char* in, size_t n, char* out, size_t cap) {
  z_stream s;
  std::memset(&s, 0, sizeof(s));
  if (inflateInit2(&s, -15) != Z_OK) return false;
  s.next_in = const_cast<unsigned char*>(in);
  s.avail_in = (uInt)n;
  s.next_out = reinterpret_cast<unsigned char*>(out);
  s.avail_out = (uInt)cap;
  const int r = inflate(&s, Z_FINISH);
  const bool ok = (r == Z_STREAM_END) && s.total_out == cap;
  inflateEnd(&s);
  return ok;
}

// all gzip members in sequence (gzip.open reads concatenated members)
bool inflate_seq(const std::vector<unsigned char>& z, std::string& out) {
  z_stream s;
  std::memset(&s, 0, sizeof(s));
  if (inflateInit2(&s, 15 + 16) != Z_OK) return false;
  out.resize(std::max<size_t>(z.size() * 4, 1 << 16));
  size_t used = 0;
  s.next_in = const_cast<unsigned char*>(z.data());
  s.avail_in = (uInt)z.size();
  for (;;) {
    if (used == out.size()) out.resize(out.size() * 2);
    s.next_out = reinterpret_cast<unsigned char*>(&out[used]);
    s.avail_out = (uInt)(out.size() - used);
    const int r = inflate(&s, Z_NO_FLUSH);
    used = out.size() - s.avail_out;
    if (r == Z_STREAM_END) {
      if (s.avail_in == 0) break;
      if (inflateReset(&s) != Z_OK) { inflateEnd(&s); return false; }
      continue;
    }
    if (r != Z_OK && !(r == Z_BUF_ERROR && s.avail_out == 0)) { inflateEnd(&s); return false; }
    if (s.avail_in == 0 && s.avail_out != 0) { inflateEnd(&s); return false; }   // truncated
  }
  inflateEnd(&s);
  out.resize(used);
  return true;
}

// ------------------------------------------------------------------------------------- lines

// Python text mode: "\n", "\r\n" and "\r" end a line; the line handed to the reference's code
// keeps one "\n" (translated) when it had a terminator.
struct Line {
  size_t b, e;      // content [b, e)
  bool nl;          // had a terminator
  size_t next;      // start of the next line
};

inline Line next_line(const char* t, size_t n, size_t p) {
  Line l;
  l.b = p;
  size_t q = p;
  while (q < n && t[q] != '\n' && t[q] != '\r') ++q;
  l.e = q;
  if (q < n) {
    l.nl = true;
    l.next = (t[q] == '\r' && q + 1 < n && t[q + 1] == '\n') ? q + 2 : q + 1;
  } else {
    l.nl = false;
    l.next = n;
  }
  return l;
}

inline bool py_space(unsigned char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0x0b || c == 0x0c || (c >= 0x1c && c <= 0x1f);
}

// ------------------------------------------------------------------------------------- records

struct Part {   // one thread's records, in file order
  std::vector<uint64_t> hash;
  std::vector<int64_t> key_off;        // key = text[key_b[i], key_e[i]) built as chrom + '-' + pos
  std::string keys;                    // concatenated keys
  std::vector<uint32_t> chrom_len;     // chrom part length within the key
  std::vector<int32_t> ann;            // local annotation ids
  std::vector<std::string> ann_names;
  std::unordered_map<std::string, int32_t> ann_ix;
  std::vector<uint8_t> alle;           // 2 per record
  std::vector<int32_t> calls;          // P*2 per record
  int64_t lines = 0;
  bool late_header = false;
  bool failed = false;
  Fail fail;
  int64_t fail_line = 0;               // line number within the chunk
};

inline uint64_t fnv(const char* s, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ (unsigned char)s[i]) * 1099511628211ull;
  return h;
}

// the threads this process may run at once: the CPUs of its affinity mask, capped by the cgroup's
// CPU quota (cpu.max) and by OMP_NUM_THREADS when set -- a container's share of a large host, not
// hardware_concurrency(), which counts every CPU of the machine
int host_threads() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, (int)CPU_COUNT(&set));
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0) {
      const long long quota = std::atoll(q);
      if (quota > 0) n = std::min<int>(n, (int)std::max<long long>(1, (quota + period - 1) / period));
    }
    std::fclose(f);
  }
  if (const char* ev = std::getenv("OMP_NUM_THREADS")) {
    const int k = std::atoi(ev);
    if (k > 0) n = std::min(n, k);
  }
  return std::max(1, n);
}

struct Ctx {
  const char* t;
  size_t n;
  std::vector<int32_t> poplist;   // population id of each mapped sample, in header order
  int P = 0;
};

// The reference's loop body for one data line (twoDSFS_class.py:87-134).  Returns false on an
// exception (p.fail set).
bool parse_record(const Ctx& C, const Line& L, Part& p, std::string& tmp, std::vector<int32_t>& cnt) {
  // the line as Python sees it: content + "\n" when it had a terminator (read in place when that
  // terminator is a "\n" already; "\r" / "\r\n" lines are copied with it translated)
  const char* s;
  size_t n;
  if (L.nl && C.t[L.e] == '\n') {
    s = C.t + L.b;
    n = L.e - L.b + 1;
  } else {
    tmp.assign(C.t + L.b, L.e - L.b);
    if (L.nl) tmp.push_back('\n');
    s = tmp.data();
    n = tmp.size();
  }
  // cols = line.split("\t"): field boundaries
  size_t fb[10], fe[10];
  int nf = 0;
  size_t q = 0;
  while (nf < 10) {
    size_t e = q;
    while (e < n && s[e] != '\t') ++e;
    fb[nf] = q;
    fe[nf] = e;
    ++nf;
    if (e >= n) break;
    q = e + 1;
  }
  const size_t samples_at = nf == 10 ? fb[9] : n + 1;   // start of cols[9:] (n+1: none)
  const int ncols = nf;                                 // (capped at 10; exact up to 9)
  auto fld = [&](int i) { return std::string_view(s + fb[i], fe[i] - fb[i]); };
  if (ncols < 8) {   // cols[7]
    p.fail = {SFS2D_VCF_E_INDEX, "IndexError: list index out of range (INFO column missing)"};
    return false;
  }
  // annotation: info.split('|')[1] when there are >= 2 parts
  const std::string_view info = fld(7);
  std::string_view annotation = "No annotation";
  const size_t bar = info.find('|');
  if (bar != std::string_view::npos) {
    const size_t bar2 = info.find('|', bar + 1);
    annotation = info.substr(bar + 1, bar2 == std::string_view::npos ? std::string_view::npos : bar2 - bar - 1);
  }
  const std::string_view filt = fld(6);
  if (filt != "PASS" && filt != ".") return true;
  auto base = [](std::string_view a) -> int {
    if (a.size() != 1) return 0;
    const char c = a[0] & ~0x20;   // upper() of an ASCII letter
    return (c == 'A' || c == 'C' || c == 'G' || c == 'T') && ((a[0] | 0x20) >= 'a' && (a[0] | 0x20) <= 'z') ? c : 0;
  };
  const int ref = base(fld(3)), alt = base(fld(4));
  if (!ref || !alt) return true;
  if (ncols < 9) {   // cols[8]
    p.fail = {SFS2D_VCF_E_INDEX, "IndexError: list index out of range (FORMAT column missing)"};
    return false;
  }
  // gtindex = cols[8].split(':').index('GT')
  const std::string_view fmt = fld(8);
  int gti = -1;
  {
    int k = 0;
    size_t a = 0;
    for (;;) {
      size_t b = fmt.find(':', a);
      const std::string_view sub = fmt.substr(a, b == std::string_view::npos ? std::string_view::npos : b - a);
      if (sub == "GT") { gti = k; break; }
      if (b == std::string_view::npos) break;
      a = b + 1;
      ++k;
    }
  }
  if (gti < 0) {
    p.fail = {SFS2D_VCF_E_VALUE, "ValueError: 'GT' is not in list"};
    return false;
  }
  // zip(poplist, cols[9:])
  std::fill(cnt.begin(), cnt.end(), -1);
  size_t sp = samples_at;
  for (size_t j = 0; j < C.poplist.size() && sp <= n; ++j) {
    size_t se = sp;
    while (se < n && s[se] != '\t') ++se;
    // gt = sample.split(':')[gtindex]
    size_t a = sp;
    for (int k = 0; k < gti; ++k) {
      while (a < se && s[a] != ':') ++a;
      if (a >= se) {
        p.fail = {SFS2D_VCF_E_INDEX, "IndexError: list index out of range (GT subfield missing in a sample)"};
        return false;
      }
      ++a;
    }
    size_t b = a;
    while (b < se && s[b] != ':') ++b;
    int r = 0, al = 0;
    for (size_t i = a; i < b; i += 2) {   // gt[::2]
      r += s[i] == '0';
      al += s[i] == '1';
    }
    const int pop = C.poplist[j];
    if (cnt[2 * pop] < 0) cnt[2 * pop] = cnt[2 * pop + 1] = 0;
    cnt[2 * pop] += r;
    cnt[2 * pop + 1] += al;
    if (se >= n) break;
    sp = se + 1;
  }
  // snp_id = '-'.join(cols[:2])
  const size_t k0 = p.keys.size();
  p.keys.append(s + fb[0], fe[0] - fb[0]);
  if (ncols >= 2) {
    p.keys.push_back('-');
    p.keys.append(s + fb[1], fe[1] - fb[1]);
  }
  p.key_off.push_back((int64_t)p.keys.size());
  p.hash.push_back(fnv(p.keys.data() + k0, p.keys.size() - k0));
  p.chrom_len.push_back(ncols >= 2 ? (uint32_t)(fe[0] - fb[0]) : UINT32_MAX);
  // local annotation id: the previous record's, a linear search over a few names, else the map
  int32_t aid = -1;
  if (!p.ann.empty() && p.ann_names[p.ann.back()] == annotation) {
    aid = p.ann.back();
  } else if (p.ann_names.size() <= 16) {
    for (size_t i = 0; i < p.ann_names.size(); ++i)
      if (p.ann_names[i] == annotation) { aid = (int32_t)i; break; }
  } else {
    auto it = p.ann_ix.find(std::string(annotation));
    if (it != p.ann_ix.end()) aid = it->second;
  }
  if (aid < 0) {
    aid = (int32_t)p.ann_names.size();
    p.ann_ix.emplace(std::string(annotation), aid);
    p.ann_names.emplace_back(annotation);
  }
  p.ann.push_back(aid);
  p.alle.push_back((uint8_t)ref);
  p.alle.push_back((uint8_t)alt);
  p.calls.insert(p.calls.end(), cnt.begin(), cnt.end());
  return true;
}

void parse_chunk(const Ctx& C, size_t b, size_t e, Part& p) {
  std::string tmp;
  std::vector<int32_t> cnt(2 * (size_t)C.P);
  p.key_off.push_back(0);
  size_t pos = b;
  while (pos < e) {
    const Line L = next_line(C.t, e, pos);
    pos = L.next;
    ++p.lines;
    if (L.e > L.b && C.t[L.b] == '#') {
      if (L.e - L.b >= 2 && C.t[L.b + 1] == '#') continue;
      p.late_header = true;   // poplist changes mid-file: the caller reruns sequentially
      return;
    }
    if (!parse_record(C, L, p, tmp, cnt)) {
      p.failed = true;
      p.fail_line = p.lines;
      return;
    }
    if (p.hash.size() == 1) {   // room for the chunk's records at the first one's line length
      const size_t est = (e - b) / std::max<size_t>(1, L.next - L.b) + 16;
      p.hash.reserve(est); p.key_off.reserve(est + 1); p.chrom_len.reserve(est); p.ann.reserve(est);
      p.alle.reserve(2 * est); p.calls.reserve(est * 2 * (size_t)C.P);
      p.keys.reserve(est * (p.keys.size() + 2));
    }
  }
}

}  // namespace

struct sfs2d_vcf {
  int64_t n = 0;
  std::vector<std::string> pops, chroms, anns;
  std::vector<int32_t> chrom, ann, calls;
  std::vector<int64_t> pos, pos_off;
  std::string pos_blob;
  std::vector<uint8_t> alleles;
  int64_t text_bytes = 0, lines = 0;
  double t_inflate = 0, t_parse = 0, t_merge = 0;
};

extern "C" {

const char* sfs2d_vcf_last_error(void) { return g_err.c_str(); }

int sfs2d_vcf_read(const char* vcf_path, const char* popmap_path, int nthreads, sfs2d_vcf** out) {
  if (!vcf_path || !popmap_path || !out) { g_err = "null argument"; return SFS2D_VCF_E_ARG; }
  *out = nullptr;
  try {
    const auto t0 = Clock::now();
    int T = nthreads > 0 ? nthreads : host_threads();
    if (T < 1) T = 1;
    // popmap (twoDSFS_class.py:57-64): line.strip().split("\t"), >= 2 columns
    std::vector<unsigned char> pmraw;
    if (!read_file(popmap_path, pmraw)) { g_err = std::string("cannot read popmap ") + popmap_path; return SFS2D_VCF_E_IO; }
    std::unordered_map<std::string, std::string> popmap;
    {
      const char* t = reinterpret_cast<const char*>(pmraw.data());
      size_t p = 0, n = pmraw.size();
      while (p < n) {
        const Line L = next_line(t, n, p);
        p = L.next;
        size_t b = L.b, e = L.e;
        while (b < e && py_space((unsigned char)t[b])) ++b;
        while (e > b && py_space((unsigned char)t[e - 1])) --e;
        std::vector<std::string> cols;
        size_t q = b;
        for (;;) {
          size_t r = q;
          while (r < e && t[r] != '\t') ++r;
          cols.emplace_back(t + q, r - q);
          if (r >= e) break;
          q = r + 1;
        }
        if (cols.size() >= 2) popmap[cols[0]] = cols[1];
      }
    }
    // the VCF text
    std::vector<unsigned char> raw;
    if (!read_file(vcf_path, raw)) { g_err = std::string("cannot read ") + vcf_path; return SFS2D_VCF_E_IO; }
    std::string text;              // a plain gzip stream's text (one sequential inflate)
    std::unique_ptr<char[]> tbuf;  // BGZF text: not zero-filled, first touched by the inflating threads
    const char* tp = reinterpret_cast<const char*>(raw.data());   // the text (plain files: the bytes read)
    size_t tn = raw.size();
    if (raw.size() >= 2 && raw[0] == 0x1f && raw[1] == 0x8b) {
      std::vector<Member> mem;
      if (bgzf_members(raw, mem)) {
        const size_t total = mem.empty() ? 0 : mem.back().out + mem.back().isize;
        tbuf.reset(new char[total ? total : 1]);
        char* const out = tbuf.get();
        std::atomic<size_t> next{0};
        std::atomic<bool> bad{false};
        auto work = [&]() {
          for (;;) {
            const size_t i = next.fetch_add(1);
            if (i >= mem.size()) return;
            const Member& m = mem[i];
            if (m.isize && !inflate_raw(&raw[m.cdata], m.clen, out + m.out, m.isize)) bad = true;
          }
        };
        std::vector<std::thread> th;
        for (int i = 1; i < T; ++i) th.emplace_back(work);
        work();
        for (auto& x : th) x.join();
        if (bad) { g_err = std::string("corrupt BGZF block in ") + vcf_path; return SFS2D_VCF_E_GZIP; }
        tp = out;
        tn = total;
      } else if (!inflate_seq(raw, text)) {
        g_err = std::string("corrupt gzip stream in ") + vcf_path;
        return SFS2D_VCF_E_GZIP;
      } else {
        tp = text.data();
        tn = text.size();
      }
      std::vector<unsigned char>().swap(raw);
    }
    const auto t1 = Clock::now();

    Ctx C;
    C.t = tp;
    C.n = tn;
    std::vector<std::string> pops;
    std::unordered_map<std::string, int32_t> pop_ix;
    auto header = [&](const Line& L) {   // header_cols = line.split(); samples [9:] found in the popmap
      const char* t = C.t;
      std::vector<std::string_view> cols;
      size_t q = L.b;
      while (q < L.e) {
        while (q < L.e && py_space((unsigned char)t[q])) ++q;
        if (q >= L.e) break;
        size_t r = q;
        while (r < L.e && !py_space((unsigned char)t[r])) ++r;
        cols.emplace_back(t + q, r - q);
        q = r;
      }
      for (size_t i = 9; i < cols.size(); ++i) {
        auto it = popmap.find(std::string(cols[i]));
        if (it == popmap.end()) continue;
        auto jt = pop_ix.find(it->second);
        int32_t id;
        if (jt == pop_ix.end()) {
          id = (int32_t)pops.size();
          pop_ix.emplace(it->second, id);
          pops.push_back(it->second);
        } else {
          id = jt->second;
        }
        C.poplist.push_back(id);
      }
    };
    // leading '#' block, sequentially
    size_t body = 0;
    int64_t head_lines = 0;
    while (body < C.n) {
      const Line L = next_line(C.t, C.n, body);
      if (!(L.e > L.b && C.t[L.b] == '#')) break;
      ++head_lines;
      if (!(L.e - L.b >= 2 && C.t[L.b + 1] == '#')) header(L);
      body = L.next;
    }
    C.P = (int)pops.size();

    // body chunks at line starts
    std::vector<size_t> cut{body};
    const size_t span = C.n - body;
    const int nchunk = span < (size_t)(1 << 20) ? 1 : std::max(1, std::min<int>(T * 4, (int)(span >> 18)));
    for (int i = 1; i < nchunk; ++i) {
      size_t c = body + span * (size_t)i / (size_t)nchunk;
      if (c <= cut.back()) c = cut.back();
      while (c < C.n && C.t[c - 1] != '\n' && C.t[c - 1] != '\r') ++c;
      if (c < C.n && C.t[c - 1] == '\r' && C.t[c] == '\n') ++c;   // never split "\r\n"
      cut.push_back(c);
    }
    cut.push_back(C.n);
    std::vector<Part> parts(cut.size() - 1);
    {
      std::atomic<size_t> next{0};
      auto work = [&]() {
        for (;;) {
          const size_t i = next.fetch_add(1);
          if (i >= parts.size()) return;
          parse_chunk(C, cut[i], cut[i + 1], parts[i]);
        }
      };
      std::vector<std::thread> th;
      for (int i = 1; i < T && i < (int)parts.size(); ++i) th.emplace_back(work);
      work();
      for (auto& x : th) x.join();
    }
    // a header line inside the body: rerun everything after the leading block sequentially, with
    // poplist growing at each '#CHROM' line (population ids keep first-appearance order)
    bool late = false;
    for (auto& p : parts) late |= p.late_header;
    if (late) {
      parts.assign(1, Part());
      Part& p = parts[0];
      std::string tmp;
      p.key_off.push_back(0);
      size_t pos = body;
      std::vector<int32_t> cnt;
      while (pos < C.n) {
        const Line L = next_line(C.t, C.n, pos);
        pos = L.next;
        ++p.lines;
        if (L.e > L.b && C.t[L.b] == '#') {
          if (!(L.e - L.b >= 2 && C.t[L.b + 1] == '#')) {
            header(L);
            if ((int)pops.size() != C.P) {   // widen the records parsed so far
              const int P2 = (int)pops.size();
              std::vector<int32_t> w;
              const size_t nr = p.calls.size() / std::max(1, 2 * C.P);
              w.assign(nr * 2 * P2, -1);
              for (size_t r = 0; r < nr; ++r)
                for (int k = 0; k < 2 * C.P; ++k) w[r * 2 * P2 + k] = p.calls[r * 2 * C.P + k];
              p.calls.swap(w);
              C.P = P2;
            }
          }
          continue;
        }
        cnt.assign(2 * (size_t)C.P, -1);
        if (!parse_record(C, L, p, tmp, cnt)) {
          p.failed = true;
          p.fail_line = p.lines;
          break;
        }
      }
      cut.assign({body, C.n});
    }
    for (size_t i = 0; i < parts.size(); ++i) {
      if (!parts[i].failed) continue;
      int64_t line = head_lines;
      for (size_t j = 0; j < i; ++j) line += parts[j].lines;
      line += parts[i].fail_line;
      g_err = parts[i].fail.msg + " (" + vcf_path + ", line " + std::to_string(line) + ")";
      return parts[i].fail.code;
    }
    const auto t2 = Clock::now();

    // dict merge in file order: a key's slot is its first record's place, its values the last
    // record's.  Keys are sharded by hash over T threads; each thread walks every record in file
    // order, keeps those of its shard in an open-addressing table of its own and marks, per record,
    // whether it is its key's first and (first records) where the key's last values are: disjoint
    // writes, no locks.  A prefix over the first-record flags (file order) then numbers the slots.
    int64_t total = 0;
    std::vector<int64_t> base(parts.size() + 1, 0);
    for (size_t pi = 0; pi < parts.size(); ++pi) base[pi + 1] = base[pi] + (int64_t)parts[pi].hash.size();
    total = base.back();
    auto rec_id = [](size_t pi, int64_t r) { return ((int64_t)pi << 40) | r; };   // (part, record)
    std::vector<int64_t> first_id, src_id;   // per slot: (part, record) of its first / last record
    // keys unique by construction (a sorted VCF, the common case): the positions are plain decimals
    // strictly increasing within each run of one chromosome, and no chromosome comes back after
    // another -- then every record is its key's first and last, and the hash merge below is skipped
    // >= 64k records per merge shard thread (SFS2D_VCF_MERGE_CHUNK overrides: the tests use tiny
    // shards; SFS2D_VCF_HASH_MERGE=1 makes them take the hash merge on sorted files too)
    int64_t chunk = 65536;
    if (const char* ev = std::getenv("SFS2D_VCF_MERGE_CHUNK")) chunk = std::max<int64_t>(1, std::atoll(ev));
    const char* hm_ev = std::getenv("SFS2D_VCF_HASH_MERGE");
    bool uniq = !(hm_ev && hm_ev[0] == '1');
    if (uniq) {
      struct Run { std::string_view chrom; int64_t lo, hi; };
      std::vector<std::vector<Run>> runs(parts.size());
      std::vector<uint8_t> ok(parts.size(), 1);
      auto scan = [&](size_t pi) {
        const Part& p = parts[pi];
        std::vector<Run>& R = runs[pi];
        for (size_t r = 0; r < p.hash.size(); ++r) {
          const char* k = p.keys.data() + p.key_off[r];
          const size_t kl = (size_t)(p.key_off[r + 1] - p.key_off[r]);
          const uint32_t cl = p.chrom_len[r];
          if (cl == UINT32_MAX || kl - cl - 1 == 0 || kl - cl - 1 > 18) { ok[pi] = 0; return; }
          int64_t x = 0;
          for (size_t i = cl + 1; i < kl; ++i) {
            if (k[i] < '0' || k[i] > '9') { ok[pi] = 0; return; }
            x = x * 10 + (k[i] - '0');
          }
          const std::string_view ch(k, cl);
          if (R.empty() || R.back().chrom != ch) R.push_back({ch, x, x});
          else if (x <= R.back().hi) { ok[pi] = 0; return; }
          else R.back().hi = x;
        }
      };
      {
        std::atomic<size_t> next{0};
        auto work = [&]() {
          for (size_t i; (i = next.fetch_add(1)) < parts.size();) scan(i);
        };
        std::vector<std::thread> th;
        for (int i = 1; i < T && i < (int)parts.size(); ++i) th.emplace_back(work);
        work();
        for (auto& x : th) x.join();
      }
      std::unordered_map<std::string_view, int> seen;
      std::string_view cur;
      int64_t hi = 0;
      bool have = false;
      for (size_t pi = 0; pi < parts.size() && uniq; ++pi) {
        uniq = ok[pi] != 0;
        for (size_t j = 0; j < runs[pi].size() && uniq; ++j) {
          const Run& q = runs[pi][j];
          if (have && q.chrom == cur) {
            uniq = q.lo > hi;
          } else {
            uniq = seen.emplace(q.chrom, 1).second;
            cur = q.chrom;
            have = true;
          }
          hi = q.hi;
        }
      }
    }
    if (uniq) {
      first_id.reserve((size_t)total);
      for (size_t pi = 0; pi < parts.size(); ++pi)
        for (int64_t r = 0; r < (int64_t)parts[pi].hash.size(); ++r) first_id.push_back(rec_id(pi, r));
      src_id = first_id;
    } else {
      std::vector<uint8_t> is_first((size_t)total, 0);
      std::vector<int64_t> last_of((size_t)total, -1);   // first records: (part, record) of the key's last record
      {
        const int S = std::max(1, std::min<int>(T, (int)std::max<int64_t>(1, total / chunk)));
        // SFS2D_VCF_MERGE_SKEW=1 (tests): every key in shard 0, the most uneven spread the hash can give
        const char* skew_ev = std::getenv("SFS2D_VCF_MERGE_SKEW");
        const bool skew = skew_ev && skew_ev[0] == '1';
        auto shard_of = [&](uint64_t h) { return skew ? 0 : (int)((h >> 40) % (uint64_t)S); };
        auto shard = [&](int t) {
          // the table is sized from this shard's own record count (>= its distinct keys), so its load
          // factor stays <= 1/2 however unevenly the hash spreads the keys over the shards
          size_t mine = 0;
          for (const Part& p : parts)
            for (const uint64_t h : p.hash) mine += shard_of(h) == t;
          size_t cap = 16;
          while (cap < (mine + 1) * 2) cap <<= 1;
          std::vector<int64_t> table(cap, -1);   // bucket -> (part, record) of the key's first record
          for (size_t pi = 0; pi < parts.size(); ++pi) {
            const Part& p = parts[pi];
            for (size_t r = 0; r < p.hash.size(); ++r) {
              const uint64_t h = p.hash[r];
              if (shard_of(h) != t) continue;
              const char* k = p.keys.data() + p.key_off[r];
              const size_t kl = (size_t)(p.key_off[r + 1] - p.key_off[r]);
              size_t bk = h & (cap - 1);
              for (;;) {
                const int64_t g = table[bk];
                if (g < 0) {
                  const int64_t gi = base[pi] + (int64_t)r;
                  table[bk] = rec_id(pi, (int64_t)r);
                  is_first[(size_t)gi] = 1;
                  last_of[(size_t)gi] = rec_id(pi, (int64_t)r);
                  break;
                }
                const size_t qp = (size_t)(g >> 40);
                const Part& q = parts[qp];
                const int64_t fr = g & ((int64_t(1) << 40) - 1);
                const size_t ql = (size_t)(q.key_off[fr + 1] - q.key_off[fr]);
                if (q.hash[fr] == h && ql == kl && std::memcmp(q.keys.data() + q.key_off[fr], k, kl) == 0) {
                  last_of[(size_t)(base[qp] + fr)] = rec_id(pi, (int64_t)r);   // dict assignment: values replaced
                  break;
                }
                bk = (bk + 1) & (cap - 1);
              }
            }
          }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < S; ++t) th.emplace_back(shard, t);
        shard(0);
        for (auto& x : th) x.join();
      }
      first_id.reserve((size_t)total);
      src_id.reserve((size_t)total);
      for (size_t pi = 0; pi < parts.size(); ++pi)
        for (int64_t r = 0; r < (int64_t)parts[pi].hash.size(); ++r)
          if (is_first[(size_t)(base[pi] + r)]) {
            first_id.push_back(rec_id(pi, r));
            src_id.push_back(last_of[(size_t)(base[pi] + r)]);
          }
      std::vector<uint8_t>().swap(is_first);
      std::vector<int64_t>().swap(last_of);
    }
    auto part_of = [](int64_t id) { return (size_t)(id >> 40); };
    auto rec_of = [](int64_t id) { return id & ((int64_t(1) << 40) - 1); };
    auto* v = new sfs2d_vcf();
    const int64_t n = (int64_t)first_id.size();
    v->n = n;
    v->pops = pops;
    const int P = C.P;
    v->chrom.resize(n); v->ann.resize(n); v->pos.resize(n); v->pos_off.resize(n + 1);
    v->alleles.resize(2 * n); v->calls.resize((size_t)n * 2 * P);
    // chromosome and annotation ids in first-appearance order over the slots (sequential; the runs of
    // one chromosome compare a string view), positions' text offsets (a prefix)
    std::unordered_map<std::string, int32_t> cix, aix;
    std::vector<std::vector<int32_t>> amap(parts.size());
    for (size_t pi = 0; pi < parts.size(); ++pi) amap[pi].resize(parts[pi].ann_names.size(), -1);
    v->pos_off[0] = 0;
    int32_t last_cid = -1;
    for (int64_t s = 0; s < n; ++s) {
      const Part& f = parts[part_of(first_id[s])];
      const int64_t fr = rec_of(first_id[s]);
      const char* k = f.keys.data() + f.key_off[fr];
      const size_t kl = (size_t)(f.key_off[fr + 1] - f.key_off[fr]);
      const uint32_t cl = f.chrom_len[fr];
      const std::string_view chv(k, cl == UINT32_MAX ? kl : cl);
      int32_t cid;
      if (last_cid >= 0 && chv == std::string_view(v->chroms[last_cid])) {   // runs of one chromosome
        cid = last_cid;
      } else {
        std::string ch(chv);
        auto ct = cix.find(ch);
        if (ct == cix.end()) {
          cid = (int32_t)v->chroms.size();
          cix.emplace(ch, cid);
          v->chroms.push_back(ch);
        } else {
          cid = ct->second;
        }
        last_cid = cid;
      }
      v->chrom[s] = cid;
      v->pos_off[s + 1] = v->pos_off[s] + (int64_t)(cl == UINT32_MAX ? 0 : kl - cl - 1);
      const size_t sp = part_of(src_id[s]);
      const Part& p = parts[sp];
      int32_t& am = amap[sp][p.ann[rec_of(src_id[s])]];
      if (am < 0) {
        const std::string& an = p.ann_names[p.ann[rec_of(src_id[s])]];
        auto at = aix.find(an);
        if (at == aix.end()) {
          am = (int32_t)v->anns.size();
          aix.emplace(an, am);
          v->anns.push_back(an);
        } else {
          am = at->second;
        }
      }
      v->ann[s] = am;
    }
    // the rest per slot, in parallel: position text and value, alleles, calls
    v->pos_blob.resize((size_t)v->pos_off[n]);
    {
      const int W = std::max(1, std::min<int>(T, (int)std::max<int64_t>(1, n / std::max<int64_t>(1, chunk / 4))));
      auto fill = [&](int t) {
        const int64_t lo = n * t / W, hi = n * (t + 1) / W;
        for (int64_t s = lo; s < hi; ++s) {
          const Part& f = parts[part_of(first_id[s])];
          const int64_t fr = rec_of(first_id[s]);
          const char* k = f.keys.data() + f.key_off[fr];
          const size_t kl = (size_t)(f.key_off[fr + 1] - f.key_off[fr]);
          const uint32_t cl = f.chrom_len[fr];
          const char* ps = cl == UINT32_MAX ? k + kl : k + cl + 1;
          const size_t pl = (size_t)(v->pos_off[s + 1] - v->pos_off[s]);
          if (pl) std::memcpy(&v->pos_blob[(size_t)v->pos_off[s]], ps, pl);
          int64_t x = 0;
          bool okp = pl > 0 && pl <= 18;
          for (size_t i = 0; okp && i < pl; ++i) {
            if (ps[i] < '0' || ps[i] > '9') okp = false;
            else x = x * 10 + (ps[i] - '0');
          }
          v->pos[s] = okp ? x : INT64_MIN;
          const Part& p = parts[part_of(src_id[s])];
          const int64_t r = rec_of(src_id[s]);
          v->alleles[2 * s] = p.alle[2 * r];
          v->alleles[2 * s + 1] = p.alle[2 * r + 1];
          std::memcpy(&v->calls[(size_t)s * 2 * P], &p.calls[(size_t)r * 2 * P], sizeof(int32_t) * 2 * P);
        }
      };
      std::vector<std::thread> th;
      for (int t = 1; t < W; ++t) th.emplace_back(fill, t);
      fill(0);
      for (auto& x : th) x.join();
    }
    v->text_bytes = (int64_t)C.n;
    for (auto& p : parts) v->lines += p.lines;
    const auto t3 = Clock::now();
    v->t_inflate = secs(t0, t1);
    v->t_parse = secs(t1, t2);
    v->t_merge = secs(t2, t3);
    *out = v;
    return SFS2D_VCF_OK;
  } catch (const std::bad_alloc&) {
    g_err = "out of memory";
    return SFS2D_VCF_E_MEM;
  } catch (const std::exception& e) {
    g_err = e.what();
    return SFS2D_VCF_E_ARG;
  }
}

void sfs2d_vcf_free(sfs2d_vcf* v) { delete v; }
int64_t sfs2d_vcf_num_records(const sfs2d_vcf* v) { return v ? v->n : 0; }
int32_t sfs2d_vcf_num_pops(const sfs2d_vcf* v) { return v ? (int32_t)v->pops.size() : 0; }
const char* sfs2d_vcf_pop_name(const sfs2d_vcf* v, int32_t i) {
  return (v && i >= 0 && i < (int32_t)v->pops.size()) ? v->pops[i].c_str() : nullptr;
}
int32_t sfs2d_vcf_num_chroms(const sfs2d_vcf* v) { return v ? (int32_t)v->chroms.size() : 0; }
const char* sfs2d_vcf_chrom_name(const sfs2d_vcf* v, int32_t i) {
  return (v && i >= 0 && i < (int32_t)v->chroms.size()) ? v->chroms[i].c_str() : nullptr;
}
int32_t sfs2d_vcf_num_annotations(const sfs2d_vcf* v) { return v ? (int32_t)v->anns.size() : 0; }
const char* sfs2d_vcf_annotation(const sfs2d_vcf* v, int32_t i) {
  return (v && i >= 0 && i < (int32_t)v->anns.size()) ? v->anns[i].c_str() : nullptr;
}

int sfs2d_vcf_columns(const sfs2d_vcf* v, const int32_t** chrom, const int64_t** pos, const char** pos_blob,
                      const int64_t** pos_off, const int32_t** ann, const uint8_t** alleles, const int32_t** calls) {
  if (!v) return SFS2D_VCF_E_ARG;
  if (chrom) *chrom = v->chrom.data();
  if (pos) *pos = v->pos.data();
  if (pos_blob) *pos_blob = v->pos_blob.data();
  if (pos_off) *pos_off = v->pos_off.data();
  if (ann) *ann = v->ann.data();
  if (alleles) *alleles = v->alleles.data();
  if (calls) *calls = v->calls.data();
  return SFS2D_VCF_OK;
}

int sfs2d_vcf_pack(const sfs2d_vcf* v, const int32_t* chrom_rank, int32_t pop1, int32_t pop2, uint32_t* counts,
                   uint32_t* pos, uint16_t* ann) {
  if (!v || !chrom_rank || !counts || !pos || !ann) return SFS2D_VCF_E_ARG;
  const int P = (int)v->pops.size();
  if (pop1 >= P || pop2 >= P || v->anns.size() > 65535) return pop1 >= P || pop2 >= P ? SFS2D_VCF_E_ARG : 1;
  const int64_t n = v->n;
  const int T = std::max(1, std::min<int>(host_threads(), (int)std::max<int64_t>(1, n / 65536)));
  std::vector<uint8_t> bad(T, 0);
  auto work = [&](int t) {
    const int64_t lo = n * t / T, hi = n * (t + 1) / T;
    for (int64_t i = lo; i < hi; ++i) {
      const int64_t x = v->pos[i];
      if (x < 0 || x > 0xffffffffll) { bad[t] = 1; return; }   // (INT64_MIN: not a plain decimal)
      if (i > 0) {   // scan order: chromosome rank non-decreasing, positions non-decreasing within one
        const int32_t r0 = chrom_rank[v->chrom[i - 1]], r1 = chrom_rank[v->chrom[i]];
        if (r1 < r0 || (r1 == r0 && v->pos[i - 1] > x)) { bad[t] = 1; return; }
      }
      uint32_t c = 0;
      const int32_t* q = &v->calls[(size_t)i * 2 * P];
      if (pop1 >= 0 && q[2 * pop1] >= 0) {
        if (q[2 * pop1] > 255 || q[2 * pop1 + 1] > 255) { bad[t] = 1; return; }
        c |= (uint32_t)q[2 * pop1] | (uint32_t)q[2 * pop1 + 1] << 8;
      }
      if (pop2 >= 0 && q[2 * pop2] >= 0) {
        if (q[2 * pop2] > 255 || q[2 * pop2 + 1] > 255) { bad[t] = 1; return; }
        c |= (uint32_t)q[2 * pop2] << 16 | (uint32_t)q[2 * pop2 + 1] << 24;
      }
      counts[i] = c;
      pos[i] = (uint32_t)x;
      ann[i] = (uint16_t)v->ann[i];
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  for (uint8_t b : bad)
    if (b) return 1;
  return SFS2D_VCF_OK;
}

int sfs2d_vcf_stats(const sfs2d_vcf* v, int64_t* text_bytes, int64_t* lines, double* t_inflate, double* t_parse,
                    double* t_merge) {
  if (!v) return SFS2D_VCF_E_ARG;
  if (text_bytes) *text_bytes = v->text_bytes;
  if (lines) *lines = v->lines;
  if (t_inflate) *t_inflate = v->t_inflate;
  if (t_parse) *t_parse = v->t_parse;
  if (t_merge) *t_merge = v->t_merge;
  return SFS2D_VCF_OK;
}

}  // extern "C"
