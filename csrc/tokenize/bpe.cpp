// Native byte-level BPE encoder + context packer (D2 / N18 in SURVEY §2).
//
// Re-implements what the finetune workflow's Go `dataset_tokenizer` step does
// (finetuner-workflow/finetune-workflow.yaml:423-479; semantics of its knobs in
// the parameter docs at :31-81): tokenize documents with a GPT-2 style
// byte-level BPE, append EOT, pack into fixed `context` windows honouring a
// boundary token (a boundary-delimited range that does not fit the remainder
// fills it and is then re-used whole to start the next context, or the next
// context is rewound to the boundary nearest `boundary_index`), keep
// `sampling`% of contexts in an alternating pattern, pad the final context,
// and write flat little-endian uint16.
//
// The vocabulary is handed over by Python as ids only: byte -> id for the 256
// byte symbols, and merges (left id, right id, merged id) in rank order, so no
// JSON or regex library is needed here. Pre-tokenisation follows the GPT-2
// pattern  's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
// exactly for ASCII; non-ASCII code points are classified by block (letters
// unless in the general punctuation / space blocks).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#define KCA_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

enum Cls { kLetter, kDigit, kSpace, kOther };

inline uint32_t decode_utf8(const unsigned char* s, int64_t n, int64_t i, int* len) {
  unsigned char c = s[i];
  if (c < 0x80) { *len = 1; return c; }
  int l = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
  if (i + l > n) { *len = 1; return c; }
  uint32_t cp = l == 2 ? (c & 0x1f) : l == 3 ? (c & 0x0f) : (c & 0x07);
  for (int k = 1; k < l; ++k) cp = (cp << 6) | (s[i + k] & 0x3f);
  *len = l;
  return cp;
}

inline Cls classify(uint32_t cp) {
  if (cp < 0x80) {
    if ((cp >= 'a' && cp <= 'z') || (cp >= 'A' && cp <= 'Z')) return kLetter;
    if (cp >= '0' && cp <= '9') return kDigit;
    if (cp == ' ' || (cp >= 9 && cp <= 13)) return kSpace;
    return kOther;
  }
  if (cp == 0x85 || cp == 0xA0 || cp == 0x1680 || (cp >= 0x2000 && cp <= 0x200A) || cp == 0x2028 ||
      cp == 0x2029 || cp == 0x202F || cp == 0x205F || cp == 0x3000)
    return kSpace;
  if ((cp >= 0x80 && cp <= 0xBF && cp != 0xAA && cp != 0xB5 && cp != 0xBA) || cp == 0xD7 || cp == 0xF7 ||
      (cp >= 0x2010 && cp <= 0x2027) || (cp >= 0x2030 && cp <= 0x205E) || (cp >= 0x3001 && cp <= 0x3003) ||
      (cp >= 0xFF01 && cp <= 0xFF0F))
    return kOther;
  if ((cp >= 0x660 && cp <= 0x669) || (cp >= 0xFF10 && cp <= 0xFF19)) return kDigit;
  return kLetter;
}

struct PairHash {
  size_t operator()(uint64_t k) const { return std::hash<uint64_t>()(k * 0x9E3779B97F4A7C15ull); }
};

struct Bpe {
  int32_t byte_id[256];
  std::unordered_map<uint64_t, std::pair<int32_t, int32_t>, PairHash> merges;  // (a,b) -> (rank, id)
  std::unordered_map<std::string, std::vector<int32_t>> cache;

  void bpe_word(const unsigned char* s, int64_t n, std::vector<int32_t>& out) {
    std::string key((const char*)s, (size_t)n);
    auto it = cache.find(key);
    if (it != cache.end()) {
      out.insert(out.end(), it->second.begin(), it->second.end());
      return;
    }
    std::vector<int32_t> w(n);
    for (int64_t i = 0; i < n; ++i) w[i] = byte_id[s[i]];
    while (w.size() > 1) {
      int best = -1;
      int32_t best_rank = INT32_MAX, best_id = -1;
      for (size_t i = 0; i + 1 < w.size(); ++i) {
        auto m = merges.find(((uint64_t)(uint32_t)w[i] << 32) | (uint32_t)w[i + 1]);
        if (m != merges.end() && m->second.first < best_rank) {
          best_rank = m->second.first;
          best_id = m->second.second;
          best = (int)i;
        }
      }
      if (best < 0) break;
      // merge every occurrence of this pair left-to-right (same as HF BPE)
      const int32_t a = w[best], b = w[best + 1];
      std::vector<int32_t> nw;
      nw.reserve(w.size());
      for (size_t i = 0; i < w.size();) {
        if (i + 1 < w.size() && w[i] == a && w[i + 1] == b) {
          nw.push_back(best_id);
          i += 2;
        } else {
          nw.push_back(w[i]);
          i += 1;
        }
      }
      w.swap(nw);
    }
    if (cache.size() < (1u << 20)) cache.emplace(std::move(key), w);
    out.insert(out.end(), w.begin(), w.end());
  }

  void encode(const unsigned char* s, int64_t n, std::vector<int32_t>& out) {
    int64_t i = 0;
    while (i < n) {
      int l0;
      const uint32_t c0 = decode_utf8(s, n, i, &l0);
      // contractions
      if (c0 == '\'' && i + 1 < n) {
        static const char* cs[] = {"s", "t", "re", "ve", "m", "ll", "d"};
        bool hit = false;
        for (const char* c : cs) {
          size_t cl = strlen(c);
          if (i + 1 + (int64_t)cl <= n && memcmp(s + i + 1, c, cl) == 0) {
            bpe_word(s + i, 1 + cl, out);
            i += 1 + cl;
            hit = true;
            break;
          }
        }
        if (hit) continue;
      }
      // optional single ' ' then a run of one class (L, N or other)
      int64_t j = i;
      if (c0 == ' ' && i + 1 < n) j = i + 1;
      int lj;
      const uint32_t cj = decode_utf8(s, n, j, &lj);
      const Cls k = classify(cj);
      if (k != kSpace) {
        int64_t e = j + lj;
        while (e < n) {
          int le;
          if (classify(decode_utf8(s, n, e, &le)) != k) break;
          e += le;
        }
        bpe_word(s + i, e - i, out);
        i = e;
        continue;
      }
      // whitespace run [i, e)
      int64_t e = i, last = i;
      while (e < n) {
        int le;
        if (classify(decode_utf8(s, n, e, &le)) != kSpace) break;
        last = e;
        e += le;
      }
      if (e == n || last == i) {
        // \s+ to end of text, or a single whitespace char before a non-space
        const int64_t stop = (e == n) ? e : (last == i ? e : last);
        bpe_word(s + i, stop - i, out);
        i = stop;
      } else {
        bpe_word(s + i, last - i, out);  // \s+(?!\S): leave the last one for the next token
        i = last;
      }
    }
  }
};

struct Packer {
  int ctx, boundary, boundary_index, pad, eot;
  double sampling;
  std::vector<int32_t> cur;
  std::vector<uint16_t> out;
  int64_t n_ctx = 0, n_kept = 0;

  void emit() {
    const bool keep = sampling >= 100.0 ||
                      (int64_t)((n_ctx + 1) * sampling / 100.0) > (int64_t)(n_ctx * sampling / 100.0);
    if (keep) {
      for (int32_t t : cur) out.push_back((uint16_t)t);
      ++n_kept;
    }
    ++n_ctx;
  }

  // next context after `cur` (full) was emitted; returns the carried-over tokens
  std::vector<int32_t> carry_after_emit() {
    std::vector<int32_t> c;
    if (boundary_index >= 0 && boundary >= 0) {
      for (int i = std::min<int>(boundary_index, (int)cur.size() - 1); i < (int)cur.size(); ++i) {
        if (cur[i] == boundary) {
          c.assign(cur.begin() + i + 1, cur.end());
          break;
        }
      }
      if ((int)c.size() >= ctx) c.clear();
    }
    return c;
  }

  void add_range(const int32_t* r, int64_t n) {
    if ((int64_t)cur.size() + n <= ctx) {
      cur.insert(cur.end(), r, r + n);
      if ((int64_t)cur.size() == ctx) {
        emit();
        cur = carry_after_emit();
      }
      return;
    }
    if (n > ctx) {  // cannot ever fit: hard split across contexts
      int64_t p = 0;
      while (p < n) {
        int64_t take = std::min<int64_t>(ctx - (int64_t)cur.size(), n - p);
        cur.insert(cur.end(), r + p, r + p + take);
        p += take;
        if ((int64_t)cur.size() == ctx) {
          emit();
          cur = carry_after_emit();
        }
      }
      return;
    }
    // fill the remainder with the head of the range, then restart with the whole range
    const int64_t rem = ctx - (int64_t)cur.size();
    cur.insert(cur.end(), r, r + rem);
    emit();
    std::vector<int32_t> c = carry_after_emit();
    if (boundary_index >= 0 && !c.empty() && (int64_t)c.size() + n <= ctx) {
      cur = c;
    } else {
      cur.clear();
    }
    cur.insert(cur.end(), r, r + n);
    if ((int64_t)cur.size() == ctx) {
      emit();
      cur = carry_after_emit();
    }
  }

  void add(const int32_t* t, int64_t n) {
    // split into boundary-terminated ranges
    int64_t s = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (t[i] == boundary) {
        add_range(t + s, i + 1 - s);
        s = i + 1;
      }
    }
    if (s < n) add_range(t + s, n - s);
  }

  void finish() {
    if (!cur.empty()) {
      while ((int)cur.size() < ctx) cur.push_back(pad);
      emit();
      cur.clear();
    }
  }
};

}  // namespace

KCA_HOST_API void* kca_bpe_new(const int32_t* byte_ids, int n_merges, const int32_t* left,
                               const int32_t* right, const int32_t* merged) {
  Bpe* b = new Bpe();
  for (int i = 0; i < 256; ++i) b->byte_id[i] = byte_ids[i];
  b->merges.reserve((size_t)n_merges * 2);
  for (int r = 0; r < n_merges; ++r) {
    const uint64_t k = ((uint64_t)(uint32_t)left[r] << 32) | (uint32_t)right[r];
    if (!b->merges.count(k)) b->merges.emplace(k, std::make_pair((int32_t)r, merged[r]));
  }
  return b;
}

KCA_HOST_API void kca_bpe_free(void* h) { delete (Bpe*)h; }

// Returns the number of ids; if > cap only the first cap are written.
KCA_HOST_API int64_t kca_bpe_encode(void* h, const char* text, int64_t len, int32_t* out, int64_t cap) {
  std::vector<int32_t> v;
  v.reserve((size_t)(len / 3 + 8));
  ((Bpe*)h)->encode((const unsigned char*)text, len, v);
  const int64_t n = (int64_t)v.size();
  if (out) memcpy(out, v.data(), sizeof(int32_t) * (size_t)std::min(n, cap));
  return n;
}

KCA_HOST_API void* kca_packer_new(int ctx, int boundary_id, int boundary_index, int pad_id, int eot_id,
                                  double sampling_pct) {
  Packer* p = new Packer();
  p->ctx = ctx;
  p->boundary = boundary_id;
  p->boundary_index = boundary_index;
  p->pad = pad_id;
  p->eot = eot_id;
  p->sampling = sampling_pct;
  return p;
}

KCA_HOST_API void kca_packer_add(void* h, const int32_t* toks, int64_t n) { ((Packer*)h)->add(toks, n); }

// Finish (pad the tail) and write the uint16 file. stats: [contexts seen, kept].
KCA_HOST_API int kca_packer_write(void* h, const char* path, int64_t* stats) {
  Packer* p = (Packer*)h;
  p->finish();
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  const size_t w = fwrite(p->out.data(), sizeof(uint16_t), p->out.size(), f);
  fclose(f);
  if (stats) {
    stats[0] = p->n_ctx;
    stats[1] = p->n_kept;
  }
  return w == p->out.size() ? 0 : 2;
}

KCA_HOST_API void kca_packer_free(void* h) { delete (Packer*)h; }
