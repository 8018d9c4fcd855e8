// Minimal, non-executing pickle decoder for the reference's HDF5 molecule records.
//
// The reference writes every molecule as pickle.dumps({'smiles', 'target', 'precomputed'})
// (src/datasets/features.py:551-564, read back by molecular.py:279-284), where 'precomputed' is
// compute_all's dict of numpy arrays (features.py:318-334). This decoder interprets the opcode
// subset those dumps use (protocols 2-5) and rebuilds the values as plain data: None / bool / int /
// float / str / bytes / list / tuple / dict, and numpy arrays and scalars from a whitelist of
// reconstructors interpreted as data (numpy[._core|.core].multiarray._reconstruct with BUILD,
// numpy.dtype, numpy[._core|.core].multiarray.scalar, numpy[._core|.core].numeric._frombuffer,
// and _codecs.encode(str, 'latin1'), protocol 2's spelling of bytes).
// Nothing is imported, called or executed: any other global, or an opcode outside the subset,
// makes decode() fail.
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace aimx_pickle {

enum class Kind { None, Bool, Int, Float, Str, Bytes, List, Tuple, Dict, Global, Dtype, Array, Mark };

struct Obj;
// Objects live in the Decoder's arena (reused record after record: no allocation once warm) and
// stay valid until its next decode(); strings and payloads are views into the pickle's bytes.
using Ref = Obj*;

struct Obj {
  Kind k = Kind::None;
  int64_t i = 0;
  double f = 0.0;
  // Str / Bytes / Global ("module\nname") / Dtype descr ("i8", "f4", ...): sp[0..sn), a view into
  // the pickle or into `own` (strings the decoder built: globals, latin-1 bytes)
  const char* sp = nullptr;
  size_t sn = 0;
  std::string own;
  char order = '<';        // Dtype byte order
  std::vector<Ref> items;  // List / Tuple; Dict: key, value, key, value, ...
  // Array
  std::string dtype;
  std::vector<int64_t> shape;
  bool fortran = false;
  Ref raw = nullptr;  // the Bytes object holding the array payload (not copied)
  std::string_view s() const { return std::string_view(sp ? sp : "", sn); }
  void set_own() {
    sp = own.data();
    sn = own.size();
  }
  const char* bytes() const { return raw ? raw->sp : nullptr; }
  int64_t nbytes() const { return raw ? (int64_t)raw->sn : 0; }

  const Obj* get(const char* key) const {  // Dict lookup by str key
    if (k != Kind::Dict) return nullptr;
    for (size_t j = 0; j + 1 < items.size(); j += 2)
      if (items[j]->k == Kind::Str && items[j]->s() == key) return items[j + 1];
    return nullptr;
  }
  int64_t numel() const {
    int64_t n = 1;
    for (int64_t d : shape) n *= d;
    return n;
  }
};

inline int itemsize(const std::string& d) {
  if (d.size() < 2) return 0;
  return std::atoi(d.c_str() + 1);
}

// Element e of a numeric array (or of a 0-d scalar) as int64 / double; false if unsupported.
inline bool elem_i64(const Obj& a, int64_t e, int64_t* out) {
  const int sz = itemsize(a.dtype);
  const char t = a.dtype.empty() ? 0 : a.dtype[0];
  if (sz <= 0 || sz > 8 || a.nbytes() < (e + 1) * sz) return false;
  unsigned char b[8];
  std::memcpy(b, a.bytes() + e * sz, sz);
  if (a.order == '>')
    for (int j = 0; j < sz / 2; ++j) std::swap(b[j], b[sz - 1 - j]);
  uint64_t u = 0;
  for (int j = sz - 1; j >= 0; --j) u = (u << 8) | b[j];
  if (t == 'i') {
    const int sh = 64 - 8 * sz;
    *out = sh ? (int64_t)(u << sh) >> sh : (int64_t)u;
  } else if (t == 'u' || t == 'b') {
    *out = (int64_t)u;
  } else if (t == 'f') {
    double v;
    if (sz == 8) {
      std::memcpy(&v, &u, 8);
    } else if (sz == 4) {
      uint32_t w = (uint32_t)u;
      float x;
      std::memcpy(&x, &w, 4);
      v = x;
    } else {
      return false;
    }
    *out = (int64_t)v;
  } else {
    return false;
  }
  return true;
}

inline bool elem_f64(const Obj& a, int64_t e, double* out) {
  const int sz = itemsize(a.dtype);
  if (!a.dtype.empty() && a.dtype[0] == 'f') {
    if (sz > 8 || a.nbytes() < (e + 1) * sz) return false;
    unsigned char b[8];
    std::memcpy(b, a.bytes() + e * sz, sz);
    if (a.order == '>')
      for (int j = 0; j < sz / 2; ++j) std::swap(b[j], b[sz - 1 - j]);
    if (sz == 8) {
      std::memcpy(out, b, 8);
      return true;
    }
    if (sz == 4) {
      float x;
      std::memcpy(&x, b, 4);
      *out = x;
      return true;
    }
    return false;
  }
  int64_t v;
  if (!elem_i64(a, e, &v)) return false;
  *out = (double)v;
  return true;
}

// Calls f(get) with get(e) -> int64 element e, specialised once per dtype (little-endian / byte
// integer arrays, the reference's int8 features and int32 hop arrays); other dtypes go through
// elem_i64. false if the array cannot be read as integers.
template <typename F>
inline bool with_ints(const Obj& a, F&& f) {
  const int sz = itemsize(a.dtype);
  if (a.dtype.size() < 2 || sz <= 0 || a.nbytes() < a.numel() * sz) return false;
  const char t = a.dtype[0];
  const char* p = a.bytes();
  if (a.order != '>' && (t == 'i' || t == 'u')) {
    switch (sz * (t == 'i' ? 1 : -1)) {
      case 1: f([p](int64_t e) { return (int64_t)(int8_t)p[e]; }); return true;
      case -1: f([p](int64_t e) { return (int64_t)(uint8_t)p[e]; }); return true;
      case 2: f([p](int64_t e) { int16_t v; std::memcpy(&v, p + 2 * e, 2); return (int64_t)v; }); return true;
      case 4: f([p](int64_t e) { int32_t v; std::memcpy(&v, p + 4 * e, 4); return (int64_t)v; }); return true;
      case -4: f([p](int64_t e) { uint32_t v; std::memcpy(&v, p + 4 * e, 4); return (int64_t)v; }); return true;
      case 8: f([p](int64_t e) { int64_t v; std::memcpy(&v, p + 8 * e, 8); return v; }); return true;
      default: break;
    }
  }
  bool ok = true;
  f([&a, &ok](int64_t e) {
    int64_t v = 0;
    if (!elem_i64(a, e, &v)) ok = false;
    return v;
  });
  return ok;
}

// Python number (Int / Bool / Float) or 0-d numeric array as double.
inline bool as_f64(const Obj* o, double* out) {
  if (!o) return false;
  switch (o->k) {
    case Kind::Int:
    case Kind::Bool: *out = (double)o->i; return true;
    case Kind::Float: *out = o->f; return true;
    case Kind::Array: return o->numel() == 1 && elem_f64(*o, 0, out);
    default: return false;
  }
}

class Decoder {
 public:
  static constexpr int64_t kMaxElems = int64_t(1) << 40;  // per array; keeps numel * itemsize < 2^63

  // Decode one pickle; returns nullptr (and sets err) on malformed input or a disallowed opcode.
  Ref decode(const uint8_t* p, size_t n, std::string* err) {
    p_ = p;
    end_ = p + n;
    used_ = 0;
    st_.clear();
    marks_.clear();
    memo_.clear();
    while (p_ < end_) {
      const uint8_t op = *p_++;
      if (op == '.') {  // STOP
        if (st_.size() != 1) return fail(err, "STOP with bad stack");
        return st_.back();
      }
      if (!step(op)) return fail(err, msg_.empty() ? "bad opcode" : msg_);
    }
    return fail(err, "truncated pickle");
  }

 private:
  const uint8_t* p_ = nullptr;
  const uint8_t* end_ = nullptr;
  std::vector<Ref> st_;
  std::vector<size_t> marks_;
  std::vector<Ref> memo_;
  std::string msg_;
  std::vector<std::unique_ptr<Obj>> arena_;
  size_t used_ = 0;

  Ref fail(std::string* err, const std::string& m) {
    if (err) *err = m;
    return nullptr;
  }
  bool need(size_t k) { return (size_t)(end_ - p_) >= k; }
  template <typename T>
  bool rd(T* v) {
    if (!need(sizeof(T))) return false;
    std::memcpy(v, p_, sizeof(T));
    p_ += sizeof(T);
    return true;
  }
  Ref mk(Kind k) {
    if (used_ == arena_.size()) arena_.push_back(std::make_unique<Obj>());
    Obj* o = arena_[used_++].get();
    o->k = k;
    o->i = 0;
    o->f = 0.0;
    o->sp = nullptr;
    o->sn = 0;
    o->own.clear();
    o->order = '<';
    o->items.clear();
    o->dtype.clear();
    o->shape.clear();
    o->fortran = false;
    o->raw = nullptr;
    return o;
  }
  bool push_str(Kind k, size_t len) {
    if (!need(len)) return false;
    auto o = mk(k);
    o->sp = (const char*)p_;
    o->sn = len;
    p_ += len;
    st_.push_back(o);
    return true;
  }
  bool pop(Ref* r) {
    if (st_.empty()) return false;
    *r = st_.back();
    st_.pop_back();
    return true;
  }
  // the stack above the innermost MARK: [*from, st_.end()) (false without a mark)
  bool mark_from(size_t* from) {
    if (marks_.empty() || marks_.back() > st_.size()) return false;
    *from = marks_.back();
    marks_.pop_back();
    return true;
  }
  bool tuple_n(size_t n) {
    if (st_.size() < n) return false;
    auto t = mk(Kind::Tuple);
    t->items.assign(st_.end() - n, st_.end());
    st_.resize(st_.size() - n);
    st_.push_back(t);
    return true;
  }
  static bool is_global(const Ref& fn, const char* np_sub, const char* name) {  // numpy[._core|.core].<sub>\n<name>
    const std::string_view g = fn->s();
    for (const char* pre : {"numpy._core.", "numpy.core."}) {
      const size_t lp = std::strlen(pre), ls = std::strlen(np_sub), ln = std::strlen(name);
      if (g.size() == lp + ls + 1 + ln && g.compare(0, lp, pre) == 0 && g.compare(lp, ls, np_sub) == 0 &&
          g[lp + ls] == '\n' && g.compare(lp + ls + 1, ln, name) == 0)
        return true;
    }
    return false;
  }
  bool reduce(const Ref& fn, const Ref& args) {
    if (fn->k != Kind::Global || args->k != Kind::Tuple) return err("REDUCE on a non-global");
    if (is_global(fn, "multiarray", "_reconstruct")) {  // ndarray.__reduce__: empty array + BUILD
      st_.push_back(mk(Kind::Array));
      return true;
    }
    const std::string_view g = fn->s();
    if (g == "_codecs\nencode") {  // protocol <= 2 bytes: _codecs.encode(str, 'latin1')
      if (args->items.size() != 2 || args->items[0]->k != Kind::Str || args->items[1]->k != Kind::Str ||
          (args->items[1]->s() != "latin1" && args->items[1]->s() != "latin-1"))
        return err("_codecs.encode args");
      auto b = mk(Kind::Bytes);
      const std::string_view u = args->items[0]->s();  // UTF-8 of code points < 256
      for (size_t j = 0; j < u.size(); ++j) {
        const unsigned char c = (unsigned char)u[j];
        if (c < 0x80) {
          b->own.push_back((char)c);
        } else if ((c & 0xE0) == 0xC0 && j + 1 < u.size() && c <= 0xC3) {
          b->own.push_back((char)(((c & 0x1F) << 6) | ((unsigned char)u[j + 1] & 0x3F)));
          ++j;
        } else {
          return err("_codecs.encode: not latin-1");
        }
      }
      b->set_own();
      st_.push_back(b);
      return true;
    }
    if (g == "numpy\ndtype") {
      if (args->items.empty() || args->items[0]->k != Kind::Str) return err("numpy.dtype args");
      auto d = mk(Kind::Dtype);
      d->sp = args->items[0]->sp;
      d->sn = args->items[0]->sn;
      d->order = d->s() == "i1" || d->s() == "u1" || d->s() == "b1" ? '|' : '<';
      st_.push_back(d);
      return true;
    }
    if (is_global(fn, "multiarray", "scalar")) {  // numpy scalar: (dtype, raw bytes)
      if (args->items.size() < 2 || args->items[0]->k != Kind::Dtype || args->items[1]->k != Kind::Bytes)
        return err("numpy scalar args");
      auto a = mk(Kind::Array);
      a->dtype = std::string(args->items[0]->s());
      a->order = args->items[0]->order;
      a->raw = args->items[1];
      if (!size_ok(*a)) return false;
      st_.push_back(a);
      return true;
    }
    if (is_global(fn, "numeric", "_frombuffer")) {  // protocol-5 arrays: (buf, dtype, shape, order)
      if (args->items.size() < 4 || args->items[0]->k != Kind::Bytes || args->items[1]->k != Kind::Dtype ||
          args->items[2]->k != Kind::Tuple)
        return err("_frombuffer args");
      auto a = mk(Kind::Array);
      a->raw = args->items[0];
      a->dtype = std::string(args->items[1]->s());
      a->order = args->items[1]->order;
      if (!set_shape(a, args->items[2])) return false;
      a->fortran = args->items[3]->k == Kind::Str && args->items[3]->s() == "F";
      if (!size_ok(*a)) return false;
      st_.push_back(a);
      return true;
    }
    return err("global not allowed: " + std::string(g));
  }
  bool build(const Ref& obj, const Ref& state) {
    if (obj->k == Kind::Dtype) {  // (version, byteorder, ...)
      if (state->k == Kind::Tuple && state->items.size() >= 2 && state->items[1]->k == Kind::Str &&
          state->items[1]->sn > 0)
        obj->order = state->items[1]->sp[0];
      return true;
    }
    if (obj->k == Kind::Array) {  // (version, shape, dtype, is_fortran, raw bytes)
      if (state->k != Kind::Tuple || state->items.size() < 5) return err("ndarray state");
      const auto& it = state->items;
      if (it[1]->k != Kind::Tuple || it[2]->k != Kind::Dtype || it[4]->k != Kind::Bytes) return err("ndarray state types");
      if (!set_shape(obj, it[1])) return false;
      obj->dtype = std::string(it[2]->s());
      obj->order = it[2]->order;
      obj->fortran = it[3]->k == Kind::Bool && it[3]->i;
      obj->raw = it[4];
      return size_ok(*obj);
    }
    return err("BUILD on an unsupported object");
  }
  bool err(const std::string& m) {
    msg_ = m;
    return false;
  }
  // shape dims from a tuple of Ints: each >= 0, the element count bounded (no overflow later in
  // numel() * itemsize); false on anything else (malformed input never reaches an allocation)
  bool set_shape(Obj* a, const Ref& tup) {
    a->shape.clear();
    int64_t n = 1;
    for (auto& d : tup->items) {
      if (d->k != Kind::Int || d->i < 0) return err("array shape");
      if (d->i > 0 && n > kMaxElems / d->i) return err("array too large");
      n *= d->i;
      a->shape.push_back(d->i);
    }
    return true;
  }
  // the payload holds exactly numel * itemsize bytes of a known dtype
  bool size_ok(const Obj& a) {
    const int sz = itemsize(a.dtype);
    if (sz <= 0 || sz > 16) return err("array dtype");
    if (a.numel() * sz != a.nbytes()) return err("array size");
    return true;
  }

  bool step(uint8_t op) {
    Ref a, b, c;
    switch (op) {
      case 0x80: {  // PROTO
        uint8_t v;
        return rd(&v);
      }
      case 0x95: {  // FRAME
        uint64_t n;
        return rd(&n);
      }
      case '}': st_.push_back(mk(Kind::Dict)); return true;
      case ']': st_.push_back(mk(Kind::List)); return true;
      case ')': st_.push_back(mk(Kind::Tuple)); return true;
      case '(': marks_.push_back(st_.size()); return true;
      case 'N': st_.push_back(mk(Kind::None)); return true;
      case 0x88:
      case 0x89: {
        auto o = mk(Kind::Bool);
        o->i = op == 0x88;
        st_.push_back(o);
        return true;
      }
      case 'K': {
        uint8_t v;
        if (!rd(&v)) return false;
        auto o = mk(Kind::Int);
        o->i = v;
        st_.push_back(o);
        return true;
      }
      case 'M': {
        uint16_t v;
        if (!rd(&v)) return false;
        auto o = mk(Kind::Int);
        o->i = v;
        st_.push_back(o);
        return true;
      }
      case 'J': {
        int32_t v;
        if (!rd(&v)) return false;
        auto o = mk(Kind::Int);
        o->i = v;
        st_.push_back(o);
        return true;
      }
      case 0x8a: {  // LONG1: little-endian two's complement, <= 8 bytes supported
        uint8_t n;
        if (!rd(&n) || n > 8 || !need(n)) return err("LONG1 too wide");
        uint64_t u = 0;
        for (int j = n - 1; j >= 0; --j) u = (u << 8) | p_[j];
        p_ += n;
        auto o = mk(Kind::Int);
        const int sh = 64 - 8 * n;
        o->i = n == 0 ? 0 : (sh ? (int64_t)(u << sh) >> sh : (int64_t)u);
        st_.push_back(o);
        return true;
      }
      case 'G': {  // BINFLOAT, big endian
        if (!need(8)) return false;
        uint64_t u = 0;
        for (int j = 0; j < 8; ++j) u = (u << 8) | p_[j];
        p_ += 8;
        auto o = mk(Kind::Float);
        std::memcpy(&o->f, &u, 8);
        st_.push_back(o);
        return true;
      }
      case 0x8c: {
        uint8_t n;
        return rd(&n) && push_str(Kind::Str, n);
      }
      case 'X': {
        uint32_t n;
        return rd(&n) && push_str(Kind::Str, n);
      }
      case 0x8d: {
        uint64_t n;
        return rd(&n) && push_str(Kind::Str, n);
      }
      case 'C': {
        uint8_t n;
        return rd(&n) && push_str(Kind::Bytes, n);
      }
      case 'B': {
        uint32_t n;
        return rd(&n) && push_str(Kind::Bytes, n);
      }
      case 0x8e:
      case 0x96: {  // BINBYTES8, BYTEARRAY8 (protocol-5 in-band array buffers)
        uint64_t n;
        return rd(&n) && push_str(Kind::Bytes, n);
      }
      case 0x94: memo_.push_back(st_.empty() ? nullptr : st_.back()); return !st_.empty();
      case 'q': {
        uint8_t i;
        if (!rd(&i) || st_.empty()) return false;
        if (memo_.size() <= i) memo_.resize(i + 1);
        memo_[i] = st_.back();
        return true;
      }
      case 'r': {
        uint32_t i;
        if (!rd(&i) || st_.empty() || i > (1u << 26)) return false;
        if (memo_.size() <= i) memo_.resize(i + 1);
        memo_[i] = st_.back();
        return true;
      }
      case 'h': {
        uint8_t i;
        if (!rd(&i) || i >= memo_.size() || !memo_[i]) return false;
        st_.push_back(memo_[i]);
        return true;
      }
      case 'j': {
        uint32_t i;
        if (!rd(&i) || i >= memo_.size() || !memo_[i]) return false;
        st_.push_back(memo_[i]);
        return true;
      }
      case 0x85: return tuple_n(1);
      case 0x86: return tuple_n(2);
      case 0x87: return tuple_n(3);
      case 't': {
        size_t m;
        if (!mark_from(&m)) return false;
        auto t = mk(Kind::Tuple);
        t->items.assign(st_.begin() + m, st_.end());
        st_.resize(m);
        st_.push_back(t);
        return true;
      }
      case 'a':  // APPEND
        if (!pop(&a) || st_.empty() || st_.back()->k != Kind::List) return false;
        st_.back()->items.push_back(a);
        return true;
      case 'e': {  // APPENDS
        size_t m;
        if (!mark_from(&m) || m == 0 || st_[m - 1]->k != Kind::List) return false;
        auto& L = st_[m - 1]->items;
        L.insert(L.end(), st_.begin() + m, st_.end());
        st_.resize(m);
        return true;
      }
      case 's':  // SETITEM
        if (!pop(&b) || !pop(&a) || st_.empty() || st_.back()->k != Kind::Dict) return false;
        st_.back()->items.push_back(a);
        st_.back()->items.push_back(b);
        return true;
      case 'u': {  // SETITEMS
        size_t m;
        if (!mark_from(&m) || ((st_.size() - m) & 1) || m == 0 || st_[m - 1]->k != Kind::Dict) return false;
        auto& D = st_[m - 1]->items;
        D.insert(D.end(), st_.begin() + m, st_.end());
        st_.resize(m);
        return true;
      }
      case 0x93:  // STACK_GLOBAL
        if (!pop(&b) || !pop(&a) || a->k != Kind::Str || b->k != Kind::Str) return false;
        c = mk(Kind::Global);
        c->own.assign(a->sp ? a->sp : "", a->sn);
        c->own.push_back('\n');
        c->own.append(b->sp ? b->sp : "", b->sn);
        c->set_own();
        st_.push_back(c);
        return true;
      case 'c': {  // GLOBAL "module\nname\n"
        const uint8_t* q = p_;
        int nl = 0;
        while (q < end_ && nl < 2) nl += (*q++ == '\n');
        if (nl < 2) return false;
        c = mk(Kind::Global);
        c->sp = (const char*)p_;
        c->sn = size_t(q - p_ - 1);
        p_ = q;
        st_.push_back(c);
        return true;
      }
      case 'R':
        if (!pop(&b) || !pop(&a)) return false;
        return reduce(a, b);
      case 'b':
        if (!pop(&b) || st_.empty()) return false;
        return build(st_.back(), b);
      case '0': return pop(&a);  // POP
      default: return err("opcode not supported: " + std::to_string(op));
    }
  }
};

}  // namespace aimx_pickle
