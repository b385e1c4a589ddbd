// SPDX-License-Identifier: MIT
// Native ADIOS2-BP4 writer (replaces libadios2 for the reference's IO.jl:37-163).
//
// ADIOS2 is not available in this environment, so the BP4 serialization is implemented here
// from the format description (ADIOS2 2.x BP4 engine, StatsLevel=1):
//   <name>.bp/data.<k>  one per writing rank ("subfile" k = rank): 64-B header, then one
//                       process group (PG) per step with the variable records + payloads
//                       (+ the attributes in the first step)
//   <name>.bp/md.0      64-B header, then per step: PG index, variable index, attribute index,
//                       merged over all ranks by rank 0
//   <name>.bp/md.idx    64-B header, then one 64-B record per step with the md.0 offsets
// Layout details are documented in docs/BP4_FORMAT.md; grayscott_amd/io/bp4.py reads it.
//
// Usage (C ABI, driven from grayscott_amd/io/bp4.py):
//   every rank: open -> define attributes/variables -> per step { begin, put..., end } -> close
//   rank 0 additionally merges every rank's step metadata (gathered by the control plane)
//   with bp4_write_metadata().
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>
#include <emmintrin.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <chrono>
#include <map>
#include <set>
#include <mutex>
#include <thread>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

// ---- BP type ids (ADIOS2 BPBase DataTypes) and characteristic ids ----------------------
enum : uint8_t {
  type_byte = 0, type_short = 1, type_integer = 2, type_long = 4, type_real = 5, type_double = 6,
  type_string = 9, type_string_array = 12, type_unsigned_byte = 50, type_unsigned_short = 51,
  type_unsigned_integer = 52, type_unsigned_long = 54,
};
enum : uint8_t {
  characteristic_value = 0, characteristic_min = 1, characteristic_max = 2,
  characteristic_offset = 3, characteristic_dimensions = 4, characteristic_var_id = 5,
  characteristic_payload_offset = 6, characteristic_file_index = 7,
  characteristic_time_index = 8, characteristic_minmax = 12,
};

size_t type_size(uint8_t t) {
  switch (t) {
    case type_byte: case type_unsigned_byte: return 1;
    case type_short: case type_unsigned_short: return 2;
    case type_integer: case type_unsigned_integer: case type_real: return 4;
    case type_long: case type_unsigned_long: case type_double: return 8;
    default: return 0;
  }
}

struct Buf {
  std::vector<char> b;
  template <typename T> void put(const T& v) {
    const char* p = reinterpret_cast<const char*>(&v);
    b.insert(b.end(), p, p + sizeof(T));
  }
  void bytes(const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    b.insert(b.end(), c, c + n);
  }
  void zeros(size_t n) { b.insert(b.end(), n, '\0'); }
  void name(const std::string& s) {
    put<uint16_t>((uint16_t)s.size());
    bytes(s.data(), s.size());
  }
  template <typename T> void patch(size_t pos, const T& v) { memcpy(&b[pos], &v, sizeof(T)); }
  size_t size() const { return b.size(); }
};

void make_header(Buf& h, char kind, bool active) {
  // bytes 0-31: readable tag, 32-35 version chars, 36 endianness, 37 BP version,
  // 38 active flag (index table), 39 minor version, 40-63 unused
  h.b.assign(64, '\0');
  const std::string tag = "ADIOS-BP v2.10.2";
  memcpy(&h.b[0], tag.data(), tag.size());
  for (size_t i = tag.size(); i < 30; ++i) h.b[i] = ' ';
  h.b[30] = ' ';
  h.b[31] = kind;  // 'D' data, 'M' metadata, 'I' index table
  h.b[32] = '2'; h.b[33] = '1'; h.b[34] = '2';
  h.b[36] = 0;     // little endian
  h.b[37] = 4;     // BP4
  h.b[38] = active ? 1 : 0;
  h.b[39] = 2;     // BP4 minor version
}

struct Attr {
  std::string name;
  uint8_t type;           // numeric type, type_string or type_string_array
  std::vector<char> data; // numeric payload
  std::vector<std::string> strings;
  bool single;
};

struct Var {
  std::string name;
  uint8_t type;
  std::vector<uint64_t> shape, start, count;  // row-major order, empty => global single value
};

// per-step record of one put
struct Block {
  int var;
  std::vector<char> charset;  // characteristic set for the index (count, length, records)
};

struct Writer {
  std::string dir;
  int rank = 0, nranks = 1, subfile = 0;
  std::string io_name;
  FILE* data = nullptr;
  FILE* md = nullptr;
  FILE* idx = nullptr;
  uint64_t data_pos = 0;
  uint64_t md_pos = 0;
  uint32_t step = 0;  // 1-based time step of the open step
  bool step_open = false;
  bool attrs_written = false;
  bool column_major = false;
  std::vector<Attr> attrs;
  std::vector<Var> vars;
  // open step
  Buf pg;               // PG in data
  size_t pg_vars_count_pos = 0;
  uint32_t pg_nvars = 0;
  uint64_t pg_start = 0;
  std::vector<Block> blocks;
  Buf step_meta;        // serialized local step metadata (returned to the caller)
  struct Async* async = nullptr;  // bp4_async_*: the native writer thread (null: none)
};

// The asynchronous output writer (bp4_async_submit / bp4_async_result): one native thread per
// writer runs queued whole steps (wait for the step's device copy, then bp4_write_step_uv), so
// no Python code runs on the writer side and the stepping thread never contends with it for the
// interpreter lock.
struct AsyncJob {
  int64_t ticket;
  int (*wait_fn)(void*);  // e.g. libgs_hip's gs_event_sync on the snapshot's "done" event
  void* wait_arg;
  int32_t var_step, step, var_u, var_v, nmm;
  const void *u, *v, *part;
};
struct AsyncResult {
  int rc;
  std::string blob_or_error;
};
struct Async {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv, done;
  std::deque<AsyncJob> q;
  std::map<int64_t, AsyncResult> results;
  std::set<int64_t> taken;  // tickets whose result was returned (a second call is an error)
  int64_t next = 0;
  bool stop = false;
  std::string last;  // the blob of the last bp4_async_result (valid until the next call)
};

// per thread: the output and checkpoint writers run their data writes on different host
// threads, and an error message must reach the thread whose call failed
thread_local std::string g_err;

void write_all(FILE* f, const void* p, size_t n) {
  if (n && fwrite(p, 1, n, f) != n) throw std::runtime_error(std::string("write failed: ") + strerror(errno));
}

void mkdir_p(const std::string& d) {
  struct stat st;
  if (stat(d.c_str(), &st) == 0) return;
  if (mkdir(d.c_str(), 0755) != 0 && errno != EEXIST)
    throw std::runtime_error("cannot create " + d + ": " + strerror(errno));
}

template <typename T>
void minmax_fold_lanes(const T* l, const T* h, int n, T& x, T& y) {
  for (int k = 0; k < n; ++k) {
    x = l[k] < x ? l[k] : x;
    y = h[k] > y ? h[k] : y;
  }
}

// Folds p[0, n) into the running extremes: x = v < x ? v : x, y = v > y ? v : y per element (a
// NaN element never wins; a NaN already in x / y stays).
template <typename T>
void minmax_fold(const T* p, uint64_t n, T& x, T& y) {
  for (uint64_t i = 0; i < n; ++i) {
    const T v = p[i];
    x = v < x ? v : x;
    y = v > y ? v : y;
  }
}

// SSE2 folds of the float / double fields: the scalar loop is one serial compare chain (~4 ns
// per element, 1 ms per 64^3 field -- most of an output step of the reference's L=64 example).
// minps(v, acc) is exactly `v < acc ? v : acc` (the second operand wins on NaN), so every lane
// and the final lane combine follow the scalar rule; four accumulator pairs hide the latency.
template <>
void minmax_fold<float>(const float* p, uint64_t n, float& x, float& y) {
  __m128 lo[4], hi[4];
  for (int k = 0; k < 4; ++k) { lo[k] = _mm_set1_ps(x); hi[k] = _mm_set1_ps(y); }
  uint64_t i = 0;
  for (; i + 16 <= n; i += 16)
    for (int k = 0; k < 4; ++k) {
      const __m128 v = _mm_loadu_ps(p + i + 4 * k);
      lo[k] = _mm_min_ps(v, lo[k]);
      hi[k] = _mm_max_ps(v, hi[k]);
    }
  alignas(16) float l[16], h[16];
  for (int k = 0; k < 4; ++k) { _mm_store_ps(l + 4 * k, lo[k]); _mm_store_ps(h + 4 * k, hi[k]); }
  minmax_fold_lanes(l, h, 16, x, y);
  for (; i < n; ++i) { const float v = p[i]; x = v < x ? v : x; y = v > y ? v : y; }
}

template <>
void minmax_fold<double>(const double* p, uint64_t n, double& x, double& y) {
  __m128d lo[4], hi[4];
  for (int k = 0; k < 4; ++k) { lo[k] = _mm_set1_pd(x); hi[k] = _mm_set1_pd(y); }
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8)
    for (int k = 0; k < 4; ++k) {
      const __m128d v = _mm_loadu_pd(p + i + 2 * k);
      lo[k] = _mm_min_pd(v, lo[k]);
      hi[k] = _mm_max_pd(v, hi[k]);
    }
  alignas(16) double l[8], h[8];
  for (int k = 0; k < 4; ++k) { _mm_store_pd(l + 2 * k, lo[k]); _mm_store_pd(h + 2 * k, hi[k]); }
  minmax_fold_lanes(l, h, 8, x, y);
  for (; i < n; ++i) { const double v = p[i]; x = v < x ? v : x; y = v > y ? v : y; }
}

template <typename T>
void minmax_range(const T* p, uint64_t n, T& a, T& b) {
  a = n ? p[0] : T(0);
  b = a;
  if (n > 1) minmax_fold(p + 1, n - 1, a, b);
}

// Block characteristics of a whole field (512 MB per array at L=512) dominated the synchronous
// checkpoint time single-threaded. Chunks are reduced in parallel from the identity element
// and combined starting at element 0 with the same comparison rule, so the result (NaN
// handling included: a NaN only wins from element 0) equals one sequential pass.
template <typename T>
void minmax_of(const void* data, uint64_t n, double& mn, double& mx) {
  const T* p = static_cast<const T*>(data);
  T a, b;
  constexpr uint64_t kChunk = uint64_t(1) << 20;
  if (n < 2 * kChunk) {
    minmax_range(p, n, a, b);
  } else {
    using L = std::numeric_limits<T>;
    const T hi0 = L::has_infinity ? L::infinity() : L::max();
    const T lo0 = L::has_infinity ? -L::infinity() : L::lowest();
    const int64_t nchunks = (int64_t)((n + kChunk - 1) / kChunk);
    std::vector<T> lo(nchunks, hi0), hi(nchunks, lo0);
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < nchunks; ++c) {
      const uint64_t i0 = (uint64_t)c * kChunk, i1 = std::min(n, i0 + kChunk);
      T x = hi0, y = lo0;
      minmax_fold(p + i0, i1 - i0, x, y);
      lo[c] = x;
      hi[c] = y;
    }
    a = p[0];
    b = p[0];
    for (int64_t c = 0; c < nchunks; ++c) {
      a = lo[c] < a ? lo[c] : a;
      b = hi[c] > b ? hi[c] : b;
    }
  }
  mn = (double)a;
  mx = (double)b;
}

void put_value_bytes(Buf& o, uint8_t type, double v) {
  switch (type) {
    case type_real: o.put<float>((float)v); break;
    case type_double: o.put<double>(v); break;
    case type_integer: o.put<int32_t>((int32_t)v); break;
    case type_long: o.put<int64_t>((int64_t)v); break;
    case type_unsigned_integer: o.put<uint32_t>((uint32_t)v); break;
    case type_unsigned_long: o.put<uint64_t>((uint64_t)v); break;
    case type_short: o.put<int16_t>((int16_t)v); break;
    case type_unsigned_short: o.put<uint16_t>((uint16_t)v); break;
    case type_byte: o.put<int8_t>((int8_t)v); break;
    case type_unsigned_byte: o.put<uint8_t>((uint8_t)v); break;
    default: throw std::runtime_error("bad type");
  }
}

// Attribute record in the data PG (written once, with the first step).
void put_attribute_in_data(Writer& w, Buf& o, const Attr& a, uint32_t id) {
  const size_t lenpos = o.size();
  o.zeros(4);
  o.put<uint32_t>(id);
  o.name(a.name);
  o.zeros(2);  // path
  o.put<char>('n');  // no associated variable
  o.bytes("[AMD", 4);
  o.put<uint8_t>(a.type);
  if (a.type == type_string) {
    o.put<uint32_t>((uint32_t)a.strings[0].size());
    o.bytes(a.strings[0].data(), a.strings[0].size());
  } else if (a.type == type_string_array) {
    o.put<uint32_t>((uint32_t)a.strings.size());
    for (auto& s : a.strings) {
      o.put<uint32_t>((uint32_t)s.size());
      o.bytes(s.data(), s.size());
    }
  } else {
    o.put<uint32_t>((uint32_t)a.data.size());
    o.bytes(a.data.data(), a.data.size());
  }
  o.bytes("AMD]", 4);
  o.patch<uint32_t>(lenpos, (uint32_t)(o.size() - lenpos));
  (void)w;
}

// Attribute index entry (metadata).
void put_attribute_index(Writer& w, Buf& o, const Attr& a, uint32_t id, uint64_t offset) {
  const size_t lenpos = o.size();
  o.zeros(4);
  o.put<uint32_t>(id);
  o.zeros(2);  // group name
  o.name(a.name);
  o.zeros(2);  // path
  o.put<uint8_t>(a.type);
  o.put<uint64_t>(1);  // characteristic sets
  const size_t cpos = o.size();
  o.zeros(5);
  uint8_t n = 0;
  o.put<uint8_t>(characteristic_time_index); o.put<uint32_t>(w.step); ++n;
  o.put<uint8_t>(characteristic_file_index); o.put<uint32_t>((uint32_t)w.subfile); ++n;
  o.put<uint8_t>(characteristic_value);
  if (a.type == type_string) {
    o.put<uint16_t>((uint16_t)a.strings[0].size());
    o.bytes(a.strings[0].data(), a.strings[0].size());
  } else if (a.type == type_string_array) {
    o.put<uint32_t>((uint32_t)a.strings.size());
    for (auto& s : a.strings) {
      o.put<uint16_t>((uint16_t)s.size());
      o.bytes(s.data(), s.size());
    }
  } else {
    const size_t ts = type_size(a.type);
    o.put<uint16_t>((uint16_t)(a.data.size() / ts));  // elements
    o.bytes(a.data.data(), a.data.size());
  }
  ++n;
  o.put<uint8_t>(characteristic_offset); o.put<uint64_t>(offset); ++n;
  o.put<uint8_t>(characteristic_payload_offset); o.put<uint64_t>(offset); ++n;
  o.patch<uint8_t>(cpos, n);
  o.patch<uint32_t>(cpos + 1, (uint32_t)(o.size() - cpos - 5));
  o.patch<uint32_t>(lenpos, (uint32_t)(o.size() - lenpos - 4));
}

}  // namespace

extern "C" {

const char* bp4_last_error(void) { return g_err.c_str(); }
int bp4_version(void) { return 4; }

// Open a writer that continues an existing output (restart with the output history kept):
// the first `steps_kept` steps stay, everything after them is cut off.  data_end: length to
// keep of this rank's data.<rank> (-1: start a new subfile); md_end / idx_end (rank 0): lengths
// to keep of md.0 / md.idx.  The lengths come from the index (grayscott_amd/io/bp4.py
// append_plan).  New steps continue the step numbering; attributes are not written again.
void* bp4_open_append(const char* path, const char* io_name, int32_t rank, int32_t nranks,
                      int32_t column_major, uint32_t steps_kept, int64_t data_end,
                      int64_t md_end, int64_t idx_end) {
  Writer* w = nullptr;
  try {
    if (steps_kept == 0) throw std::runtime_error("append needs at least one kept step");
    w = new Writer;
    w->dir = path;
    w->rank = rank;
    w->nranks = nranks;
    w->subfile = rank;
    w->io_name = io_name;
    w->column_major = column_major != 0;
    w->step = steps_kept;
    w->attrs_written = true;
    mkdir_p(w->dir);
    const std::string dname = w->dir + "/data." + std::to_string(w->subfile);
    if (data_end >= 64) {
      w->data = fopen(dname.c_str(), "r+b");
      if (!w->data) throw std::runtime_error("cannot reopen " + dname + ": " + strerror(errno));
      if (ftruncate(fileno(w->data), (off_t)data_end) != 0 || fseeko(w->data, 0, SEEK_END) != 0)
        throw std::runtime_error("cannot truncate " + dname + ": " + strerror(errno));
      w->data_pos = (uint64_t)data_end;
    } else {
      w->data = fopen(dname.c_str(), "wb");
      if (!w->data) throw std::runtime_error("cannot open " + dname + ": " + strerror(errno));
      Buf h;
      make_header(h, 'D', false);
      write_all(w->data, h.b.data(), h.size());
      w->data_pos = 64;
    }
    if (rank == 0) {
      w->md = fopen((w->dir + "/md.0").c_str(), "r+b");
      w->idx = fopen((w->dir + "/md.idx").c_str(), "r+b");
      if (!w->md || !w->idx) throw std::runtime_error("cannot reopen metadata files in " + w->dir);
      if (md_end < 64 || idx_end < 64 || ftruncate(fileno(w->md), (off_t)md_end) != 0 ||
          ftruncate(fileno(w->idx), (off_t)idx_end) != 0 || fseeko(w->md, 0, SEEK_END) != 0 ||
          fseeko(w->idx, 0, SEEK_END) != 0)
        throw std::runtime_error("cannot truncate the metadata of " + w->dir);
      w->md_pos = (uint64_t)md_end;
      const uint8_t active = 1;  // index table: writer open again
      if (pwrite(fileno(w->idx), &active, 1, 38) != 1) throw std::runtime_error("pwrite failed");
    }
    return w;
  } catch (const std::exception& e) {
    g_err = e.what();
    if (w) {
      if (w->data) fclose(w->data);
      if (w->md) fclose(w->md);
      if (w->idx) fclose(w->idx);
      delete w;
    }
    return nullptr;
  }
}

void* bp4_open(const char* path, const char* io_name, int32_t rank, int32_t nranks,
               int32_t column_major) {
  try {
    Writer* w = new Writer;
    w->dir = path;
    w->rank = rank;
    w->nranks = nranks;
    w->subfile = rank;
    w->io_name = io_name;
    w->column_major = column_major != 0;
    if (rank == 0) mkdir_p(w->dir);
    else {
      // rank 0 creates the directory; tolerate the race
      for (int i = 0; i < 200; ++i) {
        struct stat st;
        if (stat(w->dir.c_str(), &st) == 0) break;
        usleep(10000);
      }
      mkdir_p(w->dir);
    }
    const std::string dname = w->dir + "/data." + std::to_string(w->subfile);
    w->data = fopen(dname.c_str(), "wb");
    if (!w->data) throw std::runtime_error("cannot open " + dname + ": " + strerror(errno));
    Buf h;
    make_header(h, 'D', false);
    write_all(w->data, h.b.data(), h.size());
    w->data_pos = 64;
    if (rank == 0) {
      w->md = fopen((w->dir + "/md.0").c_str(), "wb");
      w->idx = fopen((w->dir + "/md.idx").c_str(), "wb");
      if (!w->md || !w->idx) throw std::runtime_error("cannot open metadata files in " + w->dir);
      make_header(h, 'M', false);
      write_all(w->md, h.b.data(), h.size());
      w->md_pos = 64;
      make_header(h, 'I', true);
      write_all(w->idx, h.b.data(), h.size());
      fflush(w->idx);
    }
    return w;
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

int bp4_define_attribute(void* h, const char* name, int32_t type, const void* data, int64_t n) {
  try {
    Writer* w = (Writer*)h;
    Attr a;
    a.name = name;
    a.type = (uint8_t)type;
    a.single = n == 1;
    if (a.type == type_string || a.type == type_string_array) {
      const char* const* s = (const char* const*)data;
      for (int64_t i = 0; i < n; ++i) a.strings.push_back(s[i]);
      if (a.type == type_string && n != 1) throw std::runtime_error("string attribute needs 1 value");
    } else {
      const size_t ts = type_size(a.type);
      if (!ts) throw std::runtime_error("bad attribute type");
      a.data.assign((const char*)data, (const char*)data + ts * n);
    }
    w->attrs.push_back(a);
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// ndims == 0: global single value.  Returns the variable id.
int bp4_define_variable(void* h, const char* name, int32_t type, int32_t ndims,
                        const uint64_t* shape, const uint64_t* start, const uint64_t* count) {
  try {
    Writer* w = (Writer*)h;
    Var v;
    v.name = name;
    v.type = (uint8_t)type;
    if (!type_size(v.type)) throw std::runtime_error("bad variable type");
    for (int i = 0; i < ndims; ++i) {
      v.shape.push_back(shape[i]);
      v.start.push_back(start[i]);
      v.count.push_back(count[i]);
    }
    w->vars.push_back(v);
    return (int)w->vars.size() - 1;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int bp4_set_selection(void* h, int32_t var, const uint64_t* start, const uint64_t* count) {
  Writer* w = (Writer*)h;
  Var& v = w->vars.at(var);
  for (size_t i = 0; i < v.count.size(); ++i) {
    v.start[i] = start[i];
    v.count[i] = count[i];
  }
  return 0;
}

int bp4_begin_step(void* h) {
  try {
    Writer* w = (Writer*)h;
    if (w->step_open) throw std::runtime_error("step already open");
    w->step += 1;
    w->step_open = true;
    w->blocks.clear();
    w->pg.b.clear();
    w->pg_nvars = 0;
    w->pg_start = w->data_pos;
    Buf& o = w->pg;
    o.zeros(8);  // PG length
    o.put<char>(w->column_major ? 'y' : 'n');
    o.name(w->io_name);
    o.zeros(4);  // coordination var
    const std::string ts = std::to_string(w->step);
    o.name(ts);
    o.put<uint32_t>(w->step);
    o.put<uint8_t>(1);   // methods count
    o.put<uint16_t>(3);  // methods length
    o.put<uint8_t>(0);   // method id (POSIX file)
    o.zeros(2);          // method params
    w->pg_vars_count_pos = o.size();
    o.zeros(12);         // vars count (4) + vars length (8)
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

static int put_block(void* h, int32_t var, const void* data, const double* given_mm);

// Appends one block of variable `var` (host memory, row-major contiguous `count`).
int bp4_put(void* h, int32_t var, const void* data) { return put_block(h, var, data, nullptr); }

// bp4_put with the block's min / max supplied by the caller (computed where the data was made,
// e.g. by the GPU snapshot kernel), so the writer does not scan the block again
int bp4_put_minmax(void* h, int32_t var, const void* data, double mn, double mx) {
  const double mm[2] = {mn, mx};
  return put_block(h, var, data, mm);
}

static int put_block(void* h, int32_t var, const void* data, const double* given_mm) {
  try {
    Writer* w = (Writer*)h;
    if (!w->step_open) throw std::runtime_error("put outside a step");
    const Var& v = w->vars.at(var);
    const size_t ts = type_size(v.type);
    uint64_t n = 1;
    for (auto c : v.count) n *= c;
    const bool single = v.count.empty();
    double mn = 0, mx = 0;
    if (given_mm && !single) {
      mn = given_mm[0];
      mx = given_mm[1];
    } else switch (v.type) {
      case type_real: minmax_of<float>(data, n, mn, mx); break;
      case type_double: minmax_of<double>(data, n, mn, mx); break;
      case type_integer: minmax_of<int32_t>(data, n, mn, mx); break;
      case type_long: minmax_of<int64_t>(data, n, mn, mx); break;
      case type_unsigned_integer: minmax_of<uint32_t>(data, n, mn, mx); break;
      case type_unsigned_long: minmax_of<uint64_t>(data, n, mn, mx); break;
      case type_short: minmax_of<int16_t>(data, n, mn, mx); break;
      case type_unsigned_short: minmax_of<uint16_t>(data, n, mn, mx); break;
      case type_byte: minmax_of<int8_t>(data, n, mn, mx); break;
      default: minmax_of<uint8_t>(data, n, mn, mx); break;
    }
    Buf& o = w->pg;
    const uint64_t var_offset = w->data_pos + o.size();  // absolute offset of the record
    const size_t lenpos = o.size();
    o.zeros(8);  // var length
    o.put<uint32_t>((uint32_t)var);  // member id
    o.name(v.name);
    o.zeros(2);  // path
    o.put<uint8_t>(v.type);
    o.put<char>('n');  // is dimension
    const uint8_t nd = (uint8_t)v.count.size();
    o.put<uint8_t>(nd);
    o.put<uint16_t>((uint16_t)(27 * nd));
    for (int d = 0; d < nd; ++d) {
      o.put<char>('n'); o.put<uint64_t>(v.count[d]);
      o.put<char>('n'); o.put<uint64_t>(v.shape[d]);
      o.put<char>('n'); o.put<uint64_t>(v.start[d]);
    }
    // characteristics in data
    const size_t cpos = o.size();
    o.zeros(5);
    uint8_t nc = 0;
    o.put<uint8_t>(characteristic_dimensions);
    o.put<uint8_t>(nd);
    o.put<uint16_t>((uint16_t)(24 * nd));
    for (int d = 0; d < nd; ++d) {
      o.put<uint64_t>(v.count[d]); o.put<uint64_t>(v.shape[d]); o.put<uint64_t>(v.start[d]);
    }
    ++nc;
    if (single) {
      o.put<uint8_t>(characteristic_value); o.bytes(data, ts); ++nc;
    } else {
      o.put<uint8_t>(characteristic_minmax); o.put<uint16_t>(1);
      put_value_bytes(o, v.type, mn); put_value_bytes(o, v.type, mx); ++nc;
    }
    o.patch<uint8_t>(cpos, nc);
    o.patch<uint32_t>(cpos + 1, (uint32_t)(o.size() - cpos - 5));
    const uint64_t payload_offset = w->data_pos + o.size();
    o.patch<uint64_t>(lenpos, (uint64_t)(o.size() - lenpos - 8 + n * ts));
    // the payload goes straight to the file (no copy of large arrays into the PG buffer):
    // flush the buffered PG prefix first
    write_all(w->data, o.b.data(), o.size());
    w->data_pos += o.size();
    // remember where the buffered part ended; patching earlier bytes is done with pwrite
    write_all(w->data, data, n * ts);
    w->data_pos += n * ts;
    o.b.clear();
    ++w->pg_nvars;
    // index characteristic set for this block
    Buf cs;
    cs.zeros(5);
    uint8_t k = 0;
    cs.put<uint8_t>(characteristic_time_index); cs.put<uint32_t>(w->step); ++k;
    cs.put<uint8_t>(characteristic_file_index); cs.put<uint32_t>((uint32_t)w->subfile); ++k;
    cs.put<uint8_t>(characteristic_dimensions); cs.put<uint8_t>(nd); cs.put<uint16_t>((uint16_t)(24 * nd));
    for (int d = 0; d < nd; ++d) {
      cs.put<uint64_t>(v.count[d]); cs.put<uint64_t>(v.shape[d]); cs.put<uint64_t>(v.start[d]);
    }
    ++k;
    if (single) {
      cs.put<uint8_t>(characteristic_value); cs.bytes(data, ts); ++k;
    } else {
      cs.put<uint8_t>(characteristic_minmax); cs.put<uint16_t>(1);
      put_value_bytes(cs, v.type, mn); put_value_bytes(cs, v.type, mx); ++k;
    }
    cs.put<uint8_t>(characteristic_offset); cs.put<uint64_t>(var_offset); ++k;
    cs.put<uint8_t>(characteristic_payload_offset); cs.put<uint64_t>(payload_offset); ++k;
    cs.patch<uint8_t>(0, k);
    cs.patch<uint32_t>(1, (uint32_t)(cs.size() - 5));
    w->blocks.push_back(Block{var, cs.b});
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// Close the step's PG in the data file and build this rank's step metadata blob:
//   u32 nattr-entries-bytes, attr index bytes, pg index entry, u32 nblocks, per block
//   {u32 var, u32 len, charset bytes}
// The blob is returned through bp4_step_metadata().
int bp4_end_step(void* h) {
  try {
    Writer* w = (Writer*)h;
    if (!w->step_open) throw std::runtime_error("no open step");
    if (w->pg.size()) {  // PG header of a step without puts
      write_all(w->data, w->pg.b.data(), w->pg.size());
      w->data_pos += w->pg.size();
      w->pg.b.clear();
    }
    // attributes (first step only), written by rank 0
    Buf at;
    Buf attr_index;
    const bool with_attrs = !w->attrs_written && w->rank == 0;
    uint64_t attrs_start = w->data_pos;
    if (with_attrs) {
      at.zeros(12);
      uint32_t id = 0;
      for (auto& a : w->attrs) {
        const uint64_t off = attrs_start + at.size();
        put_attribute_in_data(*w, at, a, id);
        put_attribute_index(*w, attr_index, a, id, off);
        ++id;
      }
      at.patch<uint32_t>(0, (uint32_t)w->attrs.size());
      at.patch<uint64_t>(4, (uint64_t)(at.size() - 12));
    } else {
      at.zeros(12);
    }
    w->attrs_written = true;
    write_all(w->data, at.b.data(), at.size());
    w->data_pos += at.size();
    // patch PG length and vars count/length with positioned writes
    fflush(w->data);
    const int fd = fileno(w->data);
    const uint64_t pg_len = w->data_pos - w->pg_start - 8;
    const uint64_t vars_len = (w->data_pos - at.size()) - (w->pg_start + w->pg_vars_count_pos) - 12;
    if (pwrite(fd, &pg_len, 8, (off_t)w->pg_start) != 8 ||
        pwrite(fd, &w->pg_nvars, 4, (off_t)(w->pg_start + w->pg_vars_count_pos)) != 4 ||
        pwrite(fd, &vars_len, 8, (off_t)(w->pg_start + w->pg_vars_count_pos + 4)) != 8)
      throw std::runtime_error("pwrite failed");
    // PG index entry
    Buf pgi;
    pgi.zeros(2);
    pgi.name(w->io_name);
    pgi.put<char>(w->column_major ? 'y' : 'n');
    pgi.put<uint32_t>((uint32_t)w->rank);
    pgi.name(std::to_string(w->step));
    pgi.put<uint32_t>(w->step);
    pgi.put<uint64_t>(w->pg_start);
    pgi.patch<uint16_t>(0, (uint16_t)(pgi.size() - 2));
    // blob
    Buf& m = w->step_meta;
    m.b.clear();
    m.put<uint32_t>((uint32_t)w->step);
    m.put<uint32_t>((uint32_t)attr_index.size());
    m.bytes(attr_index.b.data(), attr_index.size());
    m.put<uint32_t>((uint32_t)(with_attrs ? w->attrs.size() : 0));
    m.put<uint32_t>((uint32_t)pgi.size());
    m.bytes(pgi.b.data(), pgi.size());
    m.put<uint32_t>((uint32_t)w->blocks.size());
    for (auto& b : w->blocks) {
      m.put<uint32_t>((uint32_t)b.var);
      m.put<uint32_t>((uint32_t)b.charset.size());
      m.bytes(b.charset.data(), b.charset.size());
    }
    w->step_open = false;
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// One output step of the simulation stream in a single call (io/output.py's asynchronous job;
// IO.jl:82-96 begin_step, put step / U / V, end_step): the caller's thread spends the whole data
// write in native code.  part: nmm per-chunk (u min, u max, v min, v max) quadruples of the
// field type (the GPU snapshot kernel's), reduced here; nmm = 0: the blocks are scanned.
int bp4_write_step_uv(void* h, int32_t var_step, int32_t step, int32_t var_u, const void* u,
                      int32_t var_v, const void* v, const void* part, int32_t nmm) {
  try {
    Writer* w = (Writer*)h;
    if (bp4_begin_step(h) != 0) return -1;
    if (put_block(h, var_step, &step, nullptr) != 0) return -1;
    if (nmm > 0 && part) {
      double mm[4] = {HUGE_VAL, -HUGE_VAL, HUGE_VAL, -HUGE_VAL};
      const bool f64 = w->vars.at(var_u).type == type_double;
      for (int32_t i = 0; i < nmm; ++i)
        for (int j = 0; j < 4; ++j) {
          const double x = f64 ? ((const double*)part)[4 * i + j] : (double)((const float*)part)[4 * i + j];
          mm[j] = (j & 1) ? std::max(mm[j], x) : std::min(mm[j], x);
        }
      if (put_block(h, var_u, u, mm) != 0 || put_block(h, var_v, v, mm + 2) != 0) return -1;
    } else if (put_block(h, var_u, u, nullptr) != 0 || put_block(h, var_v, v, nullptr) != 0) {
      return -1;
    }
    return bp4_end_step(h);
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

static void async_loop(Writer* w) {
  Async* a = w->async;
  for (;;) {
    AsyncJob j;
    {
      std::unique_lock<std::mutex> lk(a->mu);
      a->cv.wait(lk, [&] { return a->stop || !a->q.empty(); });
      if (a->q.empty()) return;  // stop, nothing queued
      j = a->q.front();
      a->q.pop_front();
    }
    AsyncResult r{0, {}};
    if (j.wait_fn && j.wait_fn(j.wait_arg) != 0) {
      // (libgs_hip's gs_event_sync: a device error, or no completion within GS_COMM_TIMEOUT)
      r = {-1, "output step " + std::to_string(j.step) +
                   ": waiting for its device copy failed (a device error, or the copy did not "
                   "complete within GS_COMM_TIMEOUT)"};
    } else if (bp4_write_step_uv(w, j.var_step, j.step, j.var_u, j.u, j.var_v, j.v, j.part,
                                 j.nmm) != 0) {
      r = {-1, g_err};
    } else {
      r.blob_or_error.assign(w->step_meta.b.data(), w->step_meta.size());
    }
    {
      std::lock_guard<std::mutex> lk(a->mu);
      a->results[j.ticket] = std::move(r);
    }
    a->done.notify_all();
  }
}

// Queue one whole output step on the writer's native thread (started on first use); the
// arrays must stay valid until bp4_async_result returns for the ticket.  Returns the ticket.
int64_t bp4_async_submit(void* h, int (*wait_fn)(void*), void* wait_arg, int32_t var_step,
                         int32_t step, int32_t var_u, const void* u, int32_t var_v, const void* v,
                         const void* part, int32_t nmm) {
  try {
    Writer* w = (Writer*)h;
    if (!w->async) {
      w->async = new Async();
      w->async->th = std::thread(async_loop, w);
    }
    Async* a = w->async;
    std::lock_guard<std::mutex> lk(a->mu);
    const int64_t t = a->next++;
    a->q.push_back(AsyncJob{t, wait_fn, wait_arg, var_step, step, var_u, var_v, nmm, u, v, part});
    a->cv.notify_one();
    return t;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// Wait for a queued step (the caller's thread blocks; ctypes releases the GIL): 0 and its
// metadata blob at *out (valid until the next call), or -1 with the step's error.
int bp4_async_result(void* h, int64_t ticket, const char** out, int64_t* n) {
  Writer* w = (Writer*)h;
  Async* a = w->async;
  if (!a) {
    g_err = "bp4_async_result: nothing was submitted";
    return -1;
  }
  std::unique_lock<std::mutex> lk(a->mu);
  if (ticket < 0 || ticket >= a->next || a->taken.count(ticket)) {
    g_err = "bp4_async_result: unknown or already consumed ticket " + std::to_string(ticket);
    return -1;
  }
  // bounded like every other blocking wait of the runtime (GS_COMM_TIMEOUT, default 900 s): the
  // writer thread's own waits are bounded too, so only a wedged file system can reach this
  const char* e = getenv("GS_COMM_TIMEOUT");
  const double tmo = (e && atof(e) > 0.0) ? atof(e) : 900.0;
  // (a system_clock deadline: the steady_clock form lowers to pthread_cond_clockwait, which the
  // toolchain's ThreadSanitizer does not intercept -- make tsan)
  const auto until = std::chrono::system_clock::now() +
                     std::chrono::duration_cast<std::chrono::system_clock::duration>(
                         std::chrono::duration<double>(tmo + 60.0));
  if (!a->done.wait_until(lk, until, [&] { return a->results.count(ticket) != 0; })) {
    g_err = "bp4_async_result: output step still not written after " + std::to_string(tmo + 60.0) +
            " s";
    return -1;
  }
  AsyncResult r = std::move(a->results[ticket]);
  a->results.erase(ticket);
  a->taken.insert(ticket);
  lk.unlock();
  if (r.rc != 0) {
    g_err = r.blob_or_error;
    return -1;
  }
  a->last = std::move(r.blob_or_error);
  *out = a->last.data();
  *n = (int64_t)a->last.size();
  return 0;
}

static void async_stop(Writer* w) {
  if (!w->async) return;
  {
    std::lock_guard<std::mutex> lk(w->async->mu);
    w->async->stop = true;
  }
  w->async->cv.notify_all();
  if (w->async->th.joinable()) w->async->th.join();
  delete w->async;
  w->async = nullptr;
}

int64_t bp4_step_metadata(void* h, const char** out) {
  Writer* w = (Writer*)h;
  *out = w->step_meta.b.data();
  return (int64_t)w->step_meta.size();
}

// Rank 0: merge the step metadata blobs of all ranks (in rank order) into md.0 + md.idx.
int bp4_write_metadata(void* h, int32_t nblobs, const char* const* blobs, const int64_t* sizes) {
  try {
    Writer* w = (Writer*)h;
    if (w->rank != 0) throw std::runtime_error("only rank 0 writes metadata");
    struct Parsed {
      std::vector<char> attr_index;
      uint32_t nattrs = 0;
      std::vector<char> pgi;
      std::vector<std::pair<uint32_t, std::vector<char>>> blocks;
    };
    std::vector<Parsed> ps(nblobs);
    uint32_t step = 0;
    for (int r = 0; r < nblobs; ++r) {
      const char* p = blobs[r];
      const char* end = p + sizes[r];
      auto rd32 = [&](uint32_t& v) {
        if (p + 4 > end) throw std::runtime_error("truncated metadata blob");
        memcpy(&v, p, 4);
        p += 4;
      };
      uint32_t n;
      rd32(step);
      rd32(n);
      ps[r].attr_index.assign(p, p + n);
      p += n;
      rd32(ps[r].nattrs);
      rd32(n);
      ps[r].pgi.assign(p, p + n);
      p += n;
      uint32_t nb;
      rd32(nb);
      for (uint32_t i = 0; i < nb; ++i) {
        uint32_t var, len;
        rd32(var);
        rd32(len);
        ps[r].blocks.emplace_back(var, std::vector<char>(p, p + len));
        p += len;
      }
    }
    Buf md;
    // PG index: u64 count, u64 length, entries
    const uint64_t pg_index_start = w->md_pos;
    md.put<uint64_t>((uint64_t)nblobs);
    const size_t pglen_pos = md.size();
    md.zeros(8);
    for (auto& pr : ps) md.bytes(pr.pgi.data(), pr.pgi.size());
    md.patch<uint64_t>(pglen_pos, (uint64_t)(md.size() - pglen_pos - 8));
    // variable index: u32 count, u64 length, one merged entry per variable
    const uint64_t vars_index_start = w->md_pos + md.size();
    uint32_t nvars_present = 0;
    const size_t vcount_pos = md.size();
    md.zeros(12);
    for (size_t vi = 0; vi < w->vars.size(); ++vi) {
      std::vector<const std::vector<char>*> sets;
      for (auto& pr : ps)
        for (auto& b : pr.blocks)
          if (b.first == vi) sets.push_back(&b.second);
      if (sets.empty()) continue;
      ++nvars_present;
      const Var& v = w->vars[vi];
      const size_t lp = md.size();
      md.zeros(4);
      md.put<uint32_t>((uint32_t)vi);
      md.zeros(2);  // group name
      md.name(v.name);
      md.zeros(2);  // path
      md.put<uint8_t>(v.type);
      md.put<uint64_t>((uint64_t)sets.size());
      for (auto* s : sets) md.bytes(s->data(), s->size());
      md.patch<uint32_t>(lp, (uint32_t)(md.size() - lp - 4));
    }
    md.patch<uint32_t>(vcount_pos, nvars_present);
    md.patch<uint64_t>(vcount_pos + 4, (uint64_t)(md.size() - vcount_pos - 12));
    // attribute index
    const uint64_t attrs_index_start = w->md_pos + md.size();
    const size_t acount_pos = md.size();
    md.zeros(12);
    uint32_t nattr = 0;
    for (auto& pr : ps) {
      md.bytes(pr.attr_index.data(), pr.attr_index.size());
      nattr += pr.nattrs;
    }
    md.patch<uint32_t>(acount_pos, nattr);
    md.patch<uint64_t>(acount_pos + 4, (uint64_t)(md.size() - acount_pos - 12));
    write_all(w->md, md.b.data(), md.size());
    fflush(w->md);
    w->md_pos += md.size();
    // index record
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    const uint64_t rec[8] = {(uint64_t)step, 0, pg_index_start, vars_index_start,
                             attrs_index_start, w->md_pos,
                             (uint64_t)tv.tv_sec * 1000 + tv.tv_usec / 1000, 0};
    write_all(w->idx, rec, sizeof(rec));
    fflush(w->idx);
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int bp4_close(void* h) {
  Writer* w = (Writer*)h;
  if (!w) return 0;
  async_stop(w);  // (runs the queued steps first)
  int rc = 0;
  if (w->data) rc |= fclose(w->data);
  if (w->md) rc |= fclose(w->md);
  if (w->idx) {
    // mark the index table inactive (writer closed)
    fflush(w->idx);
    const uint8_t inactive = 0;
    if (pwrite(fileno(w->idx), &inactive, 1, 38) != 1) rc = -1;
    rc |= fclose(w->idx);
  }
  delete w;
  return rc;
}

int bp4_flush(void* h) {
  Writer* w = (Writer*)h;
  int rc = 0;
  if (w->data) rc |= fflush(w->data);
  return rc;
}

}  // extern "C"
