// Native trace ingestion (include/crdt_trace.h): streaming gzip inflate + one-pass JSON decode of
// the reference's editing traces into the engine's staging arrays.
//
// Replaces crdt-testdata load_testing_data (src/testdata/src/lib.rs:29-48: GzDecoder ->
// serde_json::from_reader into TestData, lib.rs:10-27).  Only the schema's shape is parsed:
//   { "startContent": str, "endContent": str, "txns": [ { "patches": [[pos, del, ins], ...], ...}, ...] }
// Other keys are skipped whatever their value (serde ignores unknown fields by default).  The
// inserted strings are kept as UTF-8 and counted in Unicode scalar values, the unit every
// position in the reference counts (ins_content.chars().count(), doc.rs:383).
#include <zlib.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "crdt_gpu.h"
#include "crdt_trace.h"

namespace crdt {
void set_last_error(const std::string& s);
}

struct crdt_trace {
  std::vector<uint32_t> counts;
  std::vector<uint32_t> patches;  // 3 per patch
  std::string text, start, end;
  uint64_t start_len = 0, end_len = 0;
};

namespace {

struct TraceError {
  std::string msg;
};

// Byte source: a gzip (or plain) file inflated in 1 MiB windows, or an in-memory buffer.
class Source {
 public:
  explicit Source(gzFile f) : f_(f), buf_(1u << 20) {}
  Source(const char* p, uint64_t n) : mem_(p), mem_n_(n) {}

  int peek() {
    if (pos_ == n_ && !refill()) return -1;
    return (unsigned char)cur()[pos_];
  }
  int get() {
    int c = peek();
    if (c >= 0) ++pos_, ++consumed_;
    return c;
  }
  uint64_t offset() const { return consumed_; }
  // Append the run of plain printable ASCII (no '"' or '\\') at the cursor to `out`, within the
  // current window; returns its length (one scalar per byte).
  uint64_t take_ascii(std::string& out) {
    if (pos_ == n_ && !refill()) return 0;
    const char* b = cur() + pos_;
    uint64_t k = 0, lim = n_ - pos_;
    while (k < lim) {
      unsigned char c = (unsigned char)b[k];
      if (c < 0x20 || c >= 0x7F || c == '"' || c == '\\') break;
      ++k;
    }
    out.append(b, k);
    pos_ += k;
    consumed_ += k;
    return k;
  }

 private:
  const char* cur() const { return mem_ ? mem_ : buf_.data(); }
  bool refill() {
    if (mem_) {
      if (n_ == mem_n_) return false;
      n_ = mem_n_;  // whole buffer is one window
      return pos_ < n_;
    }
    if (!f_) return false;
    int r = gzread(f_, buf_.data(), (unsigned)buf_.size());
    if (r < 0) {
      int errnum = 0;
      const char* m = gzerror(f_, &errnum);
      throw TraceError{std::string("inflate: ") + (m ? m : "error")};
    }
    pos_ = 0;
    n_ = (uint64_t)r;
    return r > 0;
  }

  gzFile f_ = nullptr;
  std::vector<char> buf_;
  const char* mem_ = nullptr;
  uint64_t mem_n_ = 0;
  uint64_t pos_ = 0, n_ = 0, consumed_ = 0;
};

class Parser {
 public:
  explicit Parser(Source& s) : s_(s) {}

  void parse_doc(crdt_trace& t) {
    ws();
    expect('{');
    bool seen_start = false, seen_end = false, seen_txns = false;
    if (!try_close('}')) {
      do {
        ws();
        std::string key;
        string_into(key, nullptr);
        ws();
        expect(':');
        ws();
        if (key == "startContent") {
          t.start.clear();
          string_into(t.start, &t.start_len);
          seen_start = true;
        } else if (key == "endContent") {
          t.end.clear();
          string_into(t.end, &t.end_len);
          seen_end = true;
        } else if (key == "txns") {
          txns(t);
          seen_txns = true;
        } else {
          skip_value(0);
        }
        ws();
      } while (comma_or_close('}'));
    }
    ws();
    if (s_.peek() >= 0) fail("trailing characters after the document");
    if (!seen_start || !seen_end || !seen_txns) fail("missing startContent / endContent / txns");
  }

 private:
  [[noreturn]] void fail(const std::string& m) {
    throw TraceError{m + " at byte " + std::to_string(s_.offset())};
  }
  void ws() {
    for (;;) {
      int c = s_.peek();
      if (c == ' ' || c == '\n' || c == '\r' || c == '\t')
        s_.get();
      else
        return;
    }
  }
  void expect(char ch) {
    if (s_.get() != (unsigned char)ch) fail(std::string("expected '") + ch + "'");
  }
  bool try_close(char close) {
    ws();
    if (s_.peek() == (unsigned char)close) {
      s_.get();
      return true;
    }
    return false;
  }
  // After an element: ',' -> true (another follows), close -> false.
  bool comma_or_close(char close) {
    ws();
    int c = s_.get();
    if (c == ',') return true;
    if (c == (unsigned char)close) return false;
    fail(std::string("expected ',' or '") + close + "'");
  }

  uint32_t u32_number() {
    ws();
    int c = s_.peek();
    if (c < '0' || c > '9') fail("expected a non-negative integer");
    uint64_t v = 0;
    int digits = 0;
    while ((c = s_.peek()) >= '0' && c <= '9') {
      if (digits == 1 && v == 0) fail("leading zero in integer");
      v = v * 10 + (uint64_t)(c - '0');
      if (v > 0xFFFFFFFFull) fail("integer exceeds u32");
      s_.get();
      ++digits;
    }
    if (c == '.' || c == 'e' || c == 'E') fail("expected an integer");
    return (uint32_t)v;
  }

  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out.push_back((char)cp);
    } else if (cp < 0x800) {
      out.push_back((char)(0xC0 | (cp >> 6)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back((char)(0xE0 | (cp >> 12)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      out.push_back((char)(0xF0 | (cp >> 18)));
      out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  uint32_t hex4() {
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      int c = s_.get();
      uint32_t d;
      if (c >= '0' && c <= '9')
        d = (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f')
        d = (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F')
        d = (uint32_t)(c - 'A' + 10);
      else
        fail("bad \\u escape");
      v = v * 16 + d;
    }
    return v;
  }

  // A JSON string, decoded to UTF-8 and appended to `out`; *scalars += its Unicode scalar count.
  void string_into(std::string& out, uint64_t* scalars) {
    if (s_.get() != '"') fail("expected a string");
    uint64_t n = 0;
    for (;;) {
      n += s_.take_ascii(out);
      int c = s_.get();
      if (c < 0) fail("unterminated string");
      if (c == '"') break;
      if (c < 0x20) fail("control character in string");
      if (c == '\\') {
        int e = s_.get();
        uint32_t cp;
        switch (e) {
          case '"': cp = '"'; break;
          case '\\': cp = '\\'; break;
          case '/': cp = '/'; break;
          case 'b': cp = 8; break;
          case 'f': cp = 12; break;
          case 'n': cp = 10; break;
          case 'r': cp = 13; break;
          case 't': cp = 9; break;
          case 'u': {
            cp = hex4();
            if (cp >= 0xDC00 && cp <= 0xDFFF) fail("lone trailing surrogate");
            if (cp >= 0xD800 && cp <= 0xDBFF) {
              if (s_.get() != '\\' || s_.get() != 'u') fail("lone leading surrogate");
              uint32_t lo = hex4();
              if (lo < 0xDC00 || lo > 0xDFFF) fail("invalid surrogate pair");
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            break;
          }
          default: fail("bad escape");
        }
        put_utf8(out, cp);
        ++n;
        continue;
      }
      // Raw UTF-8: validate the sequence length and continuation bytes, count one scalar.
      int extra;
      uint32_t cp;
      if (c < 0x80) {
        extra = 0, cp = (uint32_t)c;
      } else if ((c & 0xE0) == 0xC0) {
        extra = 1, cp = (uint32_t)(c & 0x1F);
      } else if ((c & 0xF0) == 0xE0) {
        extra = 2, cp = (uint32_t)(c & 0x0F);
      } else if ((c & 0xF8) == 0xF0) {
        extra = 3, cp = (uint32_t)(c & 0x07);
      } else {
        fail("invalid UTF-8");
      }
      out.push_back((char)c);
      for (int i = 0; i < extra; ++i) {
        int d = s_.get();
        if (d < 0 || (d & 0xC0) != 0x80) fail("invalid UTF-8");
        cp = (cp << 6) | (uint32_t)(d & 0x3F);
        out.push_back((char)d);
      }
      static const uint32_t kMin[4] = {0, 0x80, 0x800, 0x10000};
      if (cp < kMin[extra] || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) fail("invalid UTF-8");
      ++n;
    }
    if (scalars) *scalars += n;
  }

  // Any JSON value, discarded (serde skips unknown fields).
  void skip_value(int depth) {
    if (depth > 256) fail("nesting too deep");
    ws();
    int c = s_.peek();
    if (c == '"') {
      scratch_.clear();
      string_into(scratch_, nullptr);
    } else if (c == '{') {
      s_.get();
      if (try_close('}')) return;
      do {
        ws();
        scratch_.clear();
        string_into(scratch_, nullptr);
        ws();
        expect(':');
        skip_value(depth + 1);
      } while (comma_or_close('}'));
    } else if (c == '[') {
      s_.get();
      if (try_close(']')) return;
      do skip_value(depth + 1);
      while (comma_or_close(']'));
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      s_.get();
      while ((c = s_.peek()) >= 0 && (strchr("0123456789+-.eE", c) != nullptr)) s_.get();
    } else {
      const char* lit = c == 't' ? "true" : c == 'f' ? "false" : c == 'n' ? "null" : nullptr;
      if (!lit) fail("unexpected character");
      for (const char* p = lit; *p; ++p)
        if (s_.get() != (unsigned char)*p) fail("bad literal");
    }
  }

  void patch(crdt_trace& t) {
    ws();
    expect('[');
    uint32_t pos = u32_number();
    ws();
    expect(',');
    uint32_t del = u32_number();
    ws();
    expect(',');
    ws();
    uint64_t ins = 0;
    string_into(t.text, &ins);
    if (ins > 0xFFFFFFFFull) fail("insert too long");
    ws();
    expect(']');
    t.patches.push_back(pos);
    t.patches.push_back(del);
    t.patches.push_back((uint32_t)ins);
  }

  void txns(crdt_trace& t) {
    expect('[');
    if (try_close(']')) return;
    do {
      ws();
      expect('{');
      uint64_t before = t.patches.size();
      bool seen_patches = false;
      if (!try_close('}')) {
        do {
          ws();
          scratch_.clear();
          string_into(scratch_, nullptr);
          ws();
          expect(':');
          ws();
          if (scratch_ == "patches") {
            if (seen_patches) fail("duplicate patches");
            seen_patches = true;
            expect('[');
            if (!try_close(']')) {
              do patch(t);
              while (comma_or_close(']'));
            }
          } else {
            skip_value(0);
          }
        } while (comma_or_close('}'));
      }
      if (!seen_patches) fail("txn without patches");
      t.counts.push_back((uint32_t)((t.patches.size() - before) / 3));
    } while (comma_or_close(']'));
  }

  Source& s_;
  std::string scratch_;
};

int run(Source& src, crdt_trace** out) {
  crdt_trace* t = new crdt_trace();
  try {
    Parser p(src);
    p.parse_doc(*t);
  } catch (const TraceError& e) {
    delete t;
    crdt::set_last_error("trace: " + e.msg);
    return CRDT_E_TRACE;
  } catch (const std::bad_alloc&) {
    delete t;
    crdt::set_last_error("trace: out of memory");
    return CRDT_E_NOMEM;
  }
  *out = t;
  return CRDT_OK;
}

}  // namespace

extern "C" {

int crdt_trace_load(const char* path, crdt_trace** out) {
  if (!path || !out) return CRDT_E_ARG;
  *out = nullptr;
  gzFile f = gzopen(path, "rb");  // reads plain files transparently
  if (!f) {
    crdt::set_last_error(std::string("trace: cannot open ") + path);
    return CRDT_E_IO;
  }
  gzbuffer(f, 1u << 20);
  int rc;
  try {
    Source src(f);
    rc = run(src, out);
  } catch (const TraceError& e) {  // inflate error raised outside the parser's try
    crdt::set_last_error("trace: " + e.msg);
    rc = CRDT_E_IO;
  }
  gzclose(f);
  return rc;
}

int crdt_trace_parse(const char* json, uint64_t len, crdt_trace** out) {
  if ((!json && len) || !out) return CRDT_E_ARG;
  *out = nullptr;
  Source src(json ? json : "", len);
  return run(src, out);
}

int crdt_trace_sizes(const crdt_trace* t, uint64_t* s) {
  if (!t || !s) return CRDT_E_ARG;
  s[0] = t->counts.size();
  s[1] = t->patches.size() / 3;
  s[2] = t->text.size();
  s[3] = t->start_len;
  s[4] = t->start.size();
  s[5] = t->end_len;
  s[6] = t->end.size();
  return CRDT_OK;
}

int crdt_trace_copy(const crdt_trace* t, uint32_t* counts, uint32_t* patches3, char* text, char* start,
                    char* end) {
  if (!t) return CRDT_E_ARG;
  if (counts && !t->counts.empty()) memcpy(counts, t->counts.data(), t->counts.size() * 4);
  if (patches3 && !t->patches.empty()) memcpy(patches3, t->patches.data(), t->patches.size() * 4);
  if (text && !t->text.empty()) memcpy(text, t->text.data(), t->text.size());
  if (start && !t->start.empty()) memcpy(start, t->start.data(), t->start.size());
  if (end && !t->end.empty()) memcpy(end, t->end.data(), t->end.size());
  return CRDT_OK;
}

void crdt_trace_free(crdt_trace* t) { delete t; }

}  // extern "C"
