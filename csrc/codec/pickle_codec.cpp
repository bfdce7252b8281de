// Zero-copy pickle scanner / writer -- see pickle_codec.h.
#include <climits>
#include "pickle_codec.h"

#include <cstring>
#include <sstream>
#include <unordered_map>

namespace btn {
namespace codec {

namespace {

enum Op : uint8_t {
  MARK = '(', STOP = '.', POP = '0', POP_MARK = '1', DUP = '2', FLOAT_ = 'F', INT_ = 'I',
  BININT = 'J', BININT1 = 'K', LONG_ = 'L', BININT2 = 'M', NONE_ = 'N', PERSID = 'P',
  BINPERSID = 'Q', REDUCE = 'R', STRING = 'S', BINSTRING = 'T', SHORT_BINSTRING = 'U',
  UNICODE_ = 'V', BINUNICODE = 'X', APPEND = 'a', BUILD = 'b', GLOBAL_ = 'c', DICT_ = 'd',
  EMPTY_DICT = '}', APPENDS = 'e', GET = 'g', BINGET = 'h', INST = 'i', LONG_BINGET = 'j',
  LIST_ = 'l', EMPTY_LIST = ']', OBJ = 'o', PUT = 'p', BINPUT = 'q', LONG_BINPUT = 'r',
  SETITEM = 's', TUPLE_ = 't', EMPTY_TUPLE = ')', SETITEMS = 'u', BINFLOAT = 'G',
  PROTO = 0x80, NEWOBJ = 0x81, EXT1 = 0x82, EXT2 = 0x83, EXT4 = 0x84, TUPLE1 = 0x85,
  TUPLE2 = 0x86, TUPLE3 = 0x87, NEWTRUE = 0x88, NEWFALSE = 0x89, LONG1 = 0x8a, LONG4 = 0x8b,
  BINBYTES = 'B', SHORT_BINBYTES = 'C', SHORT_BINUNICODE = 0x8c, BINUNICODE8 = 0x8d,
  BINBYTES8 = 0x8e, EMPTY_SET = 0x8f, ADDITEMS = 0x90, FROZENSET = 0x91, NEWOBJ_EX = 0x92,
  STACK_GLOBAL = 0x93, MEMOIZE = 0x94, FRAME = 0x95, BYTEARRAY8 = 0x96, NEXT_BUFFER = 0x97,
  READONLY_BUFFER = 0x98,
};

VPtr mk(Value::Kind k) {
  auto v = std::make_shared<Value>();
  v->kind = k;
  return v;
}

bool is_reconstruct(const std::string& g) {
  return g == "numpy.core.multiarray._reconstruct" || g == "numpy._core.multiarray._reconstruct";
}
bool is_frombuffer(const std::string& g) {
  return g == "numpy.core.numeric._frombuffer" || g == "numpy._core.numeric._frombuffer";
}
bool is_scalar(const std::string& g) {
  return g == "numpy.core.multiarray.scalar" || g == "numpy._core.multiarray.scalar";
}

// numpy dtype.str for a code such as "u1"/"f8" and a byteorder char.
std::string dtype_str(const std::string& code, char bo) {
  if (code.size() < 2) throw Unsupported("dtype code " + code);
  char kind = code[0];
  std::string size = code.substr(1);
  // plain numeric dtypes only: bool, (u)int, float, complex of 1..16 bytes
  if (kind != 'b' && kind != 'i' && kind != 'u' && kind != 'f' && kind != 'c')
    throw Unsupported("dtype kind " + code);
  if (size != "1" && size != "2" && size != "4" && size != "8" && size != "16")
    throw Unsupported("dtype size " + code);
  char order = bo;
  if (size == "1" || kind == 'b') order = '|';
  else if (order == '=' || order == '|') order = '<';   // native little endian host
  return std::string(1, order) + kind + size;
}

class VM {
 public:
  VM(const uint8_t* d, size_t n) : d_(d), n_(n) {}

  VPtr run() {
    while (p_ < n_) {
      uint8_t op = d_[p_++];
      switch (op) {
        case PROTO: need(1); proto_ = d_[p_++]; break;
        case FRAME: need(8); p_ += 8; break;
        case STOP: {
          if (stack_.empty()) throw Unsupported("empty stack at STOP");
          return stack_.back();
        }
        case MARK: marks_.push_back(stack_.size()); break;
        case POP: pop(); break;
        case POP_MARK: pop_mark(); break;
        case DUP: push(top()); break;
        case NONE_: push(mk(Value::NONE)); break;
        case NEWTRUE: { auto v = mk(Value::BOOL); v->b = true; push(v); break; }
        case NEWFALSE: { auto v = mk(Value::BOOL); v->b = false; push(v); break; }
        case BININT: { need(4); int32_t x; std::memcpy(&x, d_ + p_, 4); p_ += 4; push_int(x); break; }
        case BININT1: { need(1); push_int(d_[p_++]); break; }
        case BININT2: { need(2); uint16_t x; std::memcpy(&x, d_ + p_, 2); p_ += 2; push_int(x); break; }
        case LONG1: {
          need(1);
          size_t k = d_[p_++];
          need(k);
          if (k > 8) throw Unsupported("LONG1 > 64 bit");
          int64_t x = 0;
          for (size_t i = 0; i < k; ++i) x |= int64_t(d_[p_ + i]) << (8 * i);
          if (k > 0 && k < 8 && (d_[p_ + k - 1] & 0x80)) x -= int64_t(1) << (8 * k);
          p_ += k;
          push_int(x);
          break;
        }
        case BINFLOAT: {
          need(8);
          uint64_t u = 0;
          for (int i = 0; i < 8; ++i) u = (u << 8) | d_[p_ + i];
          p_ += 8;
          auto v = mk(Value::FLOAT);
          std::memcpy(&v->f, &u, 8);
          push(v);
          break;
        }
        case SHORT_BINUNICODE: { need(1); size_t k = d_[p_++]; push_str(k); break; }
        case BINUNICODE: { need(4); uint32_t k; std::memcpy(&k, d_ + p_, 4); p_ += 4; push_str(k); break; }
        case BINUNICODE8: { need(8); uint64_t k; std::memcpy(&k, d_ + p_, 8); p_ += 8; push_str(k); break; }
        case SHORT_BINBYTES: { need(1); size_t k = d_[p_++]; push_bytes(k); break; }
        case BINBYTES: { need(4); uint32_t k; std::memcpy(&k, d_ + p_, 4); p_ += 4; push_bytes(k); break; }
        case BINBYTES8: case BYTEARRAY8: {
          need(8);
          uint64_t k;
          std::memcpy(&k, d_ + p_, 8);
          p_ += 8;
          push_bytes(k);
          if (op == BYTEARRAY8) stack_.back()->bytearray = true;
          break;
        }
        case EMPTY_DICT: push(mk(Value::DICT)); break;
        case EMPTY_LIST: push(mk(Value::LIST)); break;
        case EMPTY_TUPLE: push(mk(Value::TUPLE)); break;
        case EMPTY_SET: push(mk(Value::SET)); break;
        case TUPLE1: case TUPLE2: case TUPLE3: {
          size_t k = op - TUPLE1 + 1;
          if (stack_.size() < k) throw Unsupported("stack underflow");
          auto t = mk(Value::TUPLE);
          t->items.assign(stack_.end() - long(k), stack_.end());
          stack_.resize(stack_.size() - k);
          push(t);
          break;
        }
        case TUPLE_: case LIST_: case DICT_: {
          auto items = pop_mark();
          if (op == DICT_) {
            auto dct = mk(Value::DICT);
            dct->items = std::move(items);
            push(dct);
          } else {
            auto t = mk(op == TUPLE_ ? Value::TUPLE : Value::LIST);
            t->items = std::move(items);
            push(t);
          }
          break;
        }
        case SETITEM: {
          auto v = pop(); auto k = pop();
          auto dct = top();
          if (dct->kind != Value::DICT) throw Unsupported("SETITEM on non-dict");
          dct->items.push_back(k);
          dct->items.push_back(v);
          break;
        }
        case SETITEMS: {
          auto items = pop_mark();
          auto dct = top();
          if (dct->kind != Value::DICT || items.size() % 2) throw Unsupported("SETITEMS");
          for (auto& x : items) dct->items.push_back(x);
          break;
        }
        case APPEND: {
          auto v = pop();
          auto l = top();
          if (l->kind != Value::LIST) throw Unsupported("APPEND");
          l->items.push_back(v);
          break;
        }
        case APPENDS: {
          auto items = pop_mark();
          auto l = top();
          if (l->kind != Value::LIST) throw Unsupported("APPENDS");
          for (auto& x : items) l->items.push_back(x);
          break;
        }
        case ADDITEMS: {
          auto items = pop_mark();
          auto s = top();
          for (auto& x : items) s->items.push_back(x);
          break;
        }
        case MEMOIZE: memo_[uint32_t(memo_.size())] = top(); break;
        case BINPUT: { need(1); memo_[d_[p_++]] = top(); break; }
        case LONG_BINPUT: { need(4); uint32_t k; std::memcpy(&k, d_ + p_, 4); p_ += 4; memo_[k] = top(); break; }
        case BINGET: { need(1); push(memo_get(d_[p_++])); break; }
        case LONG_BINGET: { need(4); uint32_t k; std::memcpy(&k, d_ + p_, 4); p_ += 4; push(memo_get(k)); break; }
        case GLOBAL_: {
          std::string mod = readline(), name = readline();
          auto g = mk(Value::GLOBAL);
          g->s = mod + "." + name;
          push(g);
          break;
        }
        case STACK_GLOBAL: {
          auto name = pop(); auto mod = pop();
          if (name->kind != Value::STR || mod->kind != Value::STR) throw Unsupported("STACK_GLOBAL");
          auto g = mk(Value::GLOBAL);
          g->s = mod->s + "." + name->s;
          push(g);
          break;
        }
        case REDUCE: {
          auto args = pop(); auto fn = pop();
          push(reduce(fn, args));
          break;
        }
        case BUILD: {
          auto state = pop();
          build(top(), state);
          break;
        }
        default:
          throw Unsupported("opcode " + std::to_string(op));
      }
    }
    throw Unsupported("truncated pickle");
  }

 private:
  void need(uint64_t k) {
    // k may be a peer-supplied 64-bit length: compare against what is left,
    // never p_ + k (which wraps for k near 2^64)
    if (p_ > n_ || k > uint64_t(n_ - p_)) throw Unsupported("truncated pickle");
  }
  void push(VPtr v) { stack_.push_back(std::move(v)); }
  VPtr pop() {
    if (stack_.empty() || (!marks_.empty() && stack_.size() <= marks_.back()))
      throw Unsupported("stack underflow");
    auto v = stack_.back();
    stack_.pop_back();
    return v;
  }
  VPtr top() {
    if (stack_.empty()) throw Unsupported("stack underflow");
    return stack_.back();
  }
  std::vector<VPtr> pop_mark() {
    if (marks_.empty()) throw Unsupported("no mark");
    size_t m = marks_.back();
    marks_.pop_back();
    std::vector<VPtr> items(stack_.begin() + long(m), stack_.end());
    stack_.resize(m);
    return items;
  }
  VPtr memo_get(uint32_t k) {
    auto it = memo_.find(k);
    if (it == memo_.end()) throw Unsupported("memo miss");
    return it->second;
  }
  void push_int(int64_t x) {
    auto v = mk(Value::INT);
    v->i = x;
    push(v);
  }
  void push_str(uint64_t k) {
    need(k);
    auto v = mk(Value::STR);
    v->s.assign(reinterpret_cast<const char*>(d_ + p_), k);
    p_ += k;
    push(v);
  }
  void push_bytes(uint64_t k) {
    need(k);
    auto v = mk(Value::BYTES);
    v->off = p_;
    v->len = k;
    p_ += k;
    push(v);
  }
  std::string readline() {
    size_t s = p_;
    while (p_ < n_ && d_[p_] != '\n') ++p_;
    if (p_ >= n_) throw Unsupported("truncated GLOBAL");
    std::string r(reinterpret_cast<const char*>(d_ + s), p_ - s);
    ++p_;
    return r;
  }

  // shape x itemsize == payload length, without overflow
  static bool size_matches(const Value& a) {
    const int64_t n = a.numel();
    const size_t is = a.itemsize();
    return n >= 0 && is > 0 && uint64_t(n) <= a.len / is && uint64_t(n) * is == a.len;
  }

  static std::vector<int64_t> tuple_ints(const VPtr& t) {
    if (t->kind != Value::TUPLE) throw Unsupported("shape not a tuple");
    std::vector<int64_t> r;
    for (auto& x : t->items) {
      if (x->kind != Value::INT) throw Unsupported("shape element not int");
      if (x->i < 0) throw Unsupported("negative shape element");
      r.push_back(x->i);
    }
    return r;
  }

  VPtr reduce(const VPtr& fn, const VPtr& args) {
    if (fn->kind != Value::GLOBAL || args->kind != Value::TUPLE)
      throw Unsupported("REDUCE of non-global");
    const std::string& g = fn->s;
    if (is_reconstruct(g)) {
      auto a = mk(Value::NDARRAY);
      a->dtype = "";
      return a;
    }
    if (g == "numpy.dtype") {
      if (args->items.empty() || args->items[0]->kind != Value::STR) throw Unsupported("dtype args");
      auto d = mk(Value::DTYPE);
      d->s = args->items[0]->s;
      return d;
    }
    if (is_frombuffer(g)) {
      if (args->items.size() != 4) throw Unsupported("_frombuffer args");
      auto buf = args->items[0], dt = args->items[1], shp = args->items[2], order = args->items[3];
      if (buf->kind != Value::BYTES || dt->kind != Value::DTYPE) throw Unsupported("_frombuffer types");
      auto a = mk(Value::NDARRAY);
      a->dtype = dtype_str(dt->s, dt->byteorder);
      a->shape = tuple_ints(shp);
      a->fortran = order->kind == Value::STR && order->s == "F";
      a->off = buf->off;
      a->owned = buf->owned;
      a->len = buf->len;
      if (!size_matches(*a)) throw Unsupported("_frombuffer size mismatch");
      return a;
    }
    if (is_scalar(g)) {
      if (args->items.size() != 2 || args->items[0]->kind != Value::DTYPE ||
          args->items[1]->kind != Value::BYTES)
        throw Unsupported("scalar args");
      std::string ds = dtype_str(args->items[0]->s, args->items[0]->byteorder);
      const uint8_t* p = args->items[1]->ptr(d_);
      size_t n = args->items[1]->len;
      auto v = mk(Value::INT);
      char kind = ds[1];
      if (kind == 'f' && n == 8) { v->kind = Value::FLOAT; std::memcpy(&v->f, p, 8); }
      else if (kind == 'f' && n == 4) { float x; std::memcpy(&x, p, 4); v->kind = Value::FLOAT; v->f = x; }
      else if ((kind == 'i' || kind == 'u') && n <= 8) {
        uint64_t u = 0;
        std::memcpy(&u, p, n);
        if (kind == 'i' && n < 8 && (u >> (8 * n - 1)) & 1) u |= ~uint64_t(0) << (8 * n);
        v->i = int64_t(u);
      } else if (kind == 'b' && n == 1) { v->kind = Value::BOOL; v->b = p[0] != 0; }
      else throw Unsupported("scalar dtype " + ds);
      v->np_scalar = true;
      v->dtype = ds;
      v->off = args->items[1]->off;
      v->owned = args->items[1]->owned;
      v->len = n;
      return v;
    }
    if ((g == "_codecs.encode" || g == "codecs.encode") && args->items.size() == 2 &&
        args->items[0]->kind == Value::STR && args->items[1]->kind == Value::STR &&
        (args->items[1]->s == "latin1" || args->items[1]->s == "latin-1")) {
      // protocol 2 bytes: the text is the latin-1 decoding of the bytes,
      // stored as UTF-8 -- map every code point (< 256) back to one byte
      const std::string& t = args->items[0]->s;
      auto out = std::make_shared<Bytes>();
      out->reserve(t.size());
      for (size_t i = 0; i < t.size();) {
        const uint8_t c = uint8_t(t[i]);
        if (c < 0x80) {
          out->push_back(c);
          i += 1;
        } else if ((c & 0xE0) == 0xC0 && i + 1 < t.size() && c <= 0xC3) {
          out->push_back(uint8_t(((c & 0x1F) << 6) | (uint8_t(t[i + 1]) & 0x3F)));
          i += 2;
        } else {
          throw Unsupported("latin-1 text with a code point >= 256");
        }
      }
      auto b = mk(Value::BYTES);
      b->off = 0;
      b->len = out->size();
      b->owned = std::move(out);
      return b;
    }
    if (g == "builtins.bytearray" && args->items.size() == 1 && args->items[0]->kind == Value::BYTES) {
      auto b = std::make_shared<Value>(*args->items[0]);
      b->bytearray = true;
      return b;
    }
    throw Unsupported("REDUCE " + g);
  }

  void build(const VPtr& obj, const VPtr& state) {
    if (obj->kind == Value::DTYPE) {
      if (state->kind != Value::TUPLE || state->items.size() < 2) throw Unsupported("dtype state");
      auto bo = state->items[1];
      if (bo->kind == Value::STR && !bo->s.empty()) obj->byteorder = bo->s[0];
      if (state->items.size() > 3 && state->items[2]->kind != Value::NONE)
        throw Unsupported("structured dtype");
      return;
    }
    if (obj->kind == Value::NDARRAY) {
      if (state->kind != Value::TUPLE || state->items.size() != 5) throw Unsupported("ndarray state");
      auto shp = state->items[1], dt = state->items[2], fort = state->items[3], raw = state->items[4];
      if (dt->kind != Value::DTYPE || raw->kind != Value::BYTES) throw Unsupported("ndarray state types");
      obj->shape = tuple_ints(shp);
      obj->dtype = dtype_str(dt->s, dt->byteorder);
      obj->fortran = fort->kind == Value::BOOL && fort->b;
      obj->off = raw->off;
      obj->owned = raw->owned;
      obj->len = raw->len;
      if (!size_matches(*obj)) throw Unsupported("ndarray size mismatch");
      return;
    }
    throw Unsupported("BUILD on unsupported object");
  }

  const uint8_t* d_;
  size_t n_;
  size_t p_ = 0;
  int proto_ = 0;
  std::vector<VPtr> stack_;
  std::vector<size_t> marks_;
  std::unordered_map<uint32_t, VPtr> memo_;
};

}  // namespace

const Value* Value::get(const std::string& key) const {
  if (kind != DICT) return nullptr;
  for (size_t i = 0; i + 1 < items.size(); i += 2)
    if (items[i]->kind == STR && items[i]->s == key) return items[i + 1].get();
  return nullptr;
}

int64_t Value::numel() const {
  // -1 on a negative dimension or int64 overflow: never equal to a payload
  // length, so the size checks of the ndarray constructors reject the frame
  int64_t n = 1;
  for (auto s : shape) {
    if (s < 0 || (s > 0 && n > INT64_MAX / s)) return -1;
    n *= s;
  }
  return n;
}

size_t Value::itemsize() const {
  // dtype is "<order><kind><digits>" as built by dtype_str (validated there)
  size_t n = 0;
  if (dtype.size() < 3 || dtype.size() > 4) return 0;
  for (size_t i = 2; i < dtype.size(); ++i) {
    if (dtype[i] < '0' || dtype[i] > '9') return 0;
    n = n * 10 + size_t(dtype[i] - '0');
  }
  return n;
}

VPtr parse(const uint8_t* data, size_t n) {
  VM vm(data, n);
  auto root = vm.run();
  return root;
}

std::string describe(const Value& v) {
  std::ostringstream o;
  switch (v.kind) {
    case Value::NONE: o << "None"; break;
    case Value::BOOL: o << (v.b ? "True" : "False"); break;
    case Value::INT: o << v.i; break;
    case Value::FLOAT: o << v.f; break;
    case Value::STR: o << "'" << v.s << "'"; break;
    case Value::BYTES: o << "bytes[" << v.len << "]@" << v.off; break;
    case Value::NDARRAY: {
      o << "ndarray(" << v.dtype << ",(";
      for (auto s : v.shape) o << s << ",";
      o << "))@" << v.off;
      break;
    }
    case Value::LIST: case Value::TUPLE: case Value::SET: {
      o << (v.kind == Value::LIST ? "[" : "(");
      for (auto& x : v.items) o << describe(*x) << ",";
      o << (v.kind == Value::LIST ? "]" : ")");
      break;
    }
    case Value::DICT: {
      o << "{";
      for (size_t i = 0; i + 1 < v.items.size(); i += 2)
        o << describe(*v.items[i]) << ":" << describe(*v.items[i + 1]) << ",";
      o << "}";
      break;
    }
    default: o << "?"; break;
  }
  return o.str();
}

// --------------------------------------------------------------------------
// Writer
// --------------------------------------------------------------------------
Writer::Writer(int protocol) : protocol_(protocol) {
  if (protocol < 3 || protocol > 5) throw Unsupported("writer protocol must be 3..5");
  op(PROTO);
  op(uint8_t(protocol));
}

Writer::Writer(int protocol, Bytes&& storage) : protocol_(protocol), out_(std::move(storage)) {
  if (protocol < 3 || protocol > 5) throw Unsupported("writer protocol must be 3..5");
  out_.clear();
  op(PROTO);
  op(uint8_t(protocol));
}

void Writer::raw(const void* p, size_t n) {
  auto* b = static_cast<const uint8_t*>(p);
  out_.insert(out_.end(), b, b + n);
}
void Writer::u32le(uint32_t v) { raw(&v, 4); }
void Writer::u64le(uint64_t v) { raw(&v, 8); }

void Writer::short_str(const std::string& s) { str(s); }

void Writer::global(const std::string& mod, const std::string& name) {
  if (protocol_ >= 4) {
    str(mod);
    str(name);
    op(STACK_GLOBAL);
  } else {
    op(GLOBAL_);
    raw(mod.data(), mod.size());
    op('\n');
    raw(name.data(), name.size());
    op('\n');
  }
}

void Writer::begin_dict() {
  op(EMPTY_DICT);
  op(MARK);
  marks_.push_back(out_.size());
}
void Writer::key(const std::string& k) { str(k); }
void Writer::end_dict() {
  marks_.pop_back();
  op(SETITEMS);
}
void Writer::none() { op(NONE_); }
void Writer::boolean(bool v) { op(v ? NEWTRUE : NEWFALSE); }
void Writer::integer(int64_t v) {
  if (v >= 0 && v < 256) {
    op(BININT1);
    op(uint8_t(v));
  } else if (v >= 0 && v < 65536) {
    op(BININT2);
    uint16_t x = uint16_t(v);
    raw(&x, 2);
  } else if (v >= INT32_MIN && v <= INT32_MAX) {
    op(BININT);
    int32_t x = int32_t(v);
    raw(&x, 4);
  } else {
    op(LONG1);
    op(8);
    raw(&v, 8);
  }
}
void Writer::real(double v) {
  op(BINFLOAT);
  uint64_t u;
  std::memcpy(&u, &v, 8);
  for (int i = 7; i >= 0; --i) op(uint8_t((u >> (8 * i)) & 0xff));
}
void Writer::str(const std::string& v) {
  if (v.size() < 256 && protocol_ >= 4) {
    op(SHORT_BINUNICODE);
    op(uint8_t(v.size()));
  } else {
    op(BINUNICODE);
    u32le(uint32_t(v.size()));
  }
  raw(v.data(), v.size());
}
void Writer::bytes(const void* p, size_t n) {
  if (n < 256) {
    op(SHORT_BINBYTES);
    op(uint8_t(n));
  } else if (n <= 0xffffffffu) {
    op(BINBYTES);
    u32le(uint32_t(n));
  } else {
    if (protocol_ < 4) throw Unsupported("bytes > 4GiB need protocol 4");
    op(BINBYTES8);
    u64le(n);
  }
  if (p) raw(p, n);
  else out_.resize(out_.size() + n);
}
void Writer::begin_tuple() {
  op(MARK);
  marks_.push_back(out_.size());
}
void Writer::end_tuple() {
  marks_.pop_back();
  op(TUPLE_);
}
void Writer::begin_list() {
  op(EMPTY_LIST);
  op(MARK);
  marks_.push_back(out_.size());
}
void Writer::end_list() {
  marks_.pop_back();
  op(APPENDS);
}

size_t Writer::ndarray(const std::string& code, const std::vector<int64_t>& shape, const void* data, size_t align) {
  size_t item = size_t(std::stoul(code.substr(1)));
  char bo = (item == 1 || code[0] == 'b') ? '|' : '<';
  size_t n = item;
  for (auto s : shape) n *= size_t(s);
  global("numpy.core.multiarray", "_reconstruct");
  global("numpy", "ndarray");
  integer(0);
  op(TUPLE1);
  bytes("b", 1);
  op(TUPLE3);
  op(REDUCE);
  op(MARK);
  integer(1);
  if (shape.size() >= 1 && shape.size() <= 3) {
    for (auto s : shape) integer(s);
    op(uint8_t(TUPLE1 + shape.size() - 1));
  } else {
    op(MARK);
    for (auto s : shape) integer(s);
    op(TUPLE_);
  }
  global("numpy", "dtype");
  str(code);
  op(NEWFALSE);
  op(NEWTRUE);
  op(TUPLE3);
  op(REDUCE);
  op(MARK);
  integer(3);
  str(std::string(1, bo));
  op(NONE_);
  op(NONE_);
  op(NONE_);
  integer(-1);
  integer(-1);
  integer(0);
  op(TUPLE_);
  op(BUILD);
  op(NEWFALSE);
  if (align > 1) {
    const size_t hdr = n < 256 ? 2 : (n <= 0xffffffffu ? 5 : 9);
    size_t pad = (align - (out_.size() + hdr) % align) % align;
    if (pad == 1) pad += align;                 // 1 byte is not expressible; 2a + 3b covers the rest
    if (pad % 2) {
      op(BININT1), op(0), op(POP);              // 3-byte no-op
      pad -= 3;
    }
    for (; pad; pad -= 2) op(NONE_), op(POP);   // 2-byte no-op
  }
  bytes(nullptr, n);
  size_t payload = out_.size() - n;
  if (data) std::memcpy(out_.data() + payload, data, n);
  op(TUPLE_);
  op(BUILD);
  return payload;
}

Bytes& Writer::finish() {
  op(STOP);
  return out_;
}

// --------------------------------------------------------------------------
// .btr header
// --------------------------------------------------------------------------
std::vector<uint8_t> btr_header(const std::vector<int64_t>& offsets) {
  std::vector<uint8_t> o;
  auto put = [&](const void* p, size_t n) {
    auto* b = static_cast<const uint8_t*>(p);
    o.insert(o.end(), b, b + n);
  };
  auto s = [&](const char* t) { put(t, std::strlen(t)); };
  auto binput = [&](uint8_t k) { o.push_back(BINPUT); o.push_back(k); };
  auto integer = [&](int64_t v) {
    if (v >= 0 && v < 256) { o.push_back(BININT1); o.push_back(uint8_t(v)); }
    else if (v >= 0 && v < 65536) { o.push_back(BININT2); uint16_t x = uint16_t(v); put(&x, 2); }
    else { o.push_back(BININT); int32_t x = int32_t(v); put(&x, 4); }
  };
  auto binunicode = [&](const char* t) {
    o.push_back(BINUNICODE);
    uint32_t n = uint32_t(std::strlen(t));
    put(&n, 4);
    s(t);
  };
  o.push_back(PROTO); o.push_back(3);
  o.push_back(GLOBAL_); s("numpy.core.multiarray\n_reconstruct\n"); binput(0);
  o.push_back(GLOBAL_); s("numpy\nndarray\n"); binput(1);
  integer(0); o.push_back(TUPLE1); binput(2);
  o.push_back(SHORT_BINBYTES); o.push_back(1); o.push_back('b'); binput(3);
  o.push_back(TUPLE3); binput(4);
  o.push_back(REDUCE); binput(5);
  o.push_back(MARK);
  integer(1);
  integer(int64_t(offsets.size())); o.push_back(TUPLE1); binput(6);
  o.push_back(GLOBAL_); s("numpy\ndtype\n"); binput(7);
  binunicode("i8"); binput(8);
  o.push_back(NEWFALSE); o.push_back(NEWTRUE); o.push_back(TUPLE3); binput(9);
  o.push_back(REDUCE); binput(10);
  o.push_back(MARK);
  integer(3); binunicode("<"); binput(11);
  o.push_back(NONE_); o.push_back(NONE_); o.push_back(NONE_);
  { o.push_back(BININT); int32_t m1 = -1; put(&m1, 4); }
  { o.push_back(BININT); int32_t m1 = -1; put(&m1, 4); }
  integer(0);
  o.push_back(TUPLE_); binput(12);
  o.push_back(BUILD);
  o.push_back(NEWFALSE);
  size_t nb = offsets.size() * 8;
  if (nb < 256) { o.push_back(SHORT_BINBYTES); o.push_back(uint8_t(nb)); }
  else { o.push_back(BINBYTES); uint32_t x = uint32_t(nb); put(&x, 4); }
  put(offsets.data(), nb);
  binput(13);
  o.push_back(TUPLE_); binput(14);
  o.push_back(BUILD);
  o.push_back(STOP);
  return o;
}

}  // namespace codec
}  // namespace btn
