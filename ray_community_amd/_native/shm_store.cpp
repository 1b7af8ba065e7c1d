// Shared-memory object store (the framework's Plasma equivalent; reference:
// src/ray/object_manager/plasma/{store,object_lifecycle_manager,dlmalloc}.cc).
//
// Design (single node, many processes):
//   * ONE POSIX shm segment per session, mapped by every process of the node. Readers do not
//     RPC: the object table lives inside the segment, guarded by a robust process-shared mutex,
//     so get() is a hash lookup + pin, and the payload is handed to Python as a zero-copy buffer.
//   * Layout: [Header][Entry table (open addressing, tombstones)][data arena].
//   * Arena allocator: boundary-tagged blocks, first-fit free list with immediate coalescing,
//     64-B alignment (16-B vector loads / DMA friendly, cache-line separated objects).
//   * Lifetime: create -> (writer fills) -> seal -> get/pin ... release; delete frees at once when
//     unpinned, otherwise the LAST release frees it (deferred delete). LRU tick on every get lets
//     the head pick spill victims among sealed, unpinned objects.
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace py = pybind11;

static constexpr uint64_t kMagic = 0x52434153484d5354ull;  // "RCASHMST"
static constexpr int kIdLen = 32;
static constexpr uint64_t kAlign = 64;

enum EntryState : uint32_t { EMPTY = 0, CREATED = 1, SEALED = 2, TOMBSTONE = 3 };

struct Entry {
  uint8_t id[kIdLen];
  uint32_t state;
  uint32_t id_len;
  uint64_t offset;  // payload offset from segment base
  uint64_t size;
  int64_t pins;
  uint64_t lru;
  uint32_t delete_pending;
  uint32_t pad;
};

// Block header inside the arena (boundary tags).
struct Block {
  uint64_t size;       // total block size including header, multiple of kAlign
  uint64_t prev_size;  // size of the physically previous block (0 for the first)
  uint64_t free;       // 1 = free
  uint64_t next_free;  // offsets (from arena start) in the free list, ~0 = none
  uint64_t prev_free;
  uint64_t pad[3];
};
static_assert(sizeof(Block) == kAlign, "block header must be one alignment unit");

struct Header {
  uint64_t magic;
  uint64_t total_size;
  uint64_t table_offset;
  uint64_t table_cap;
  uint64_t arena_offset;
  uint64_t arena_size;
  uint64_t free_head;  // arena-relative offset of first free block, ~0 none
  uint64_t used_bytes;
  uint64_t num_objects;
  uint64_t lru_clock;
  uint64_t num_tombstones;
  pthread_mutex_t mu;
};

static constexpr uint64_t kNone = ~0ull;

static uint64_t hash_id(const uint8_t* id, int n) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < n; ++i) {
    h ^= id[i];
    h *= 1099511628211ull;
  }
  return h;
}

class Lock {
 public:
  explicit Lock(pthread_mutex_t* m) : m_(m) {
    int rc = pthread_mutex_lock(m_);
    if (rc == EOWNERDEAD) pthread_mutex_consistent(m_);  // a process died holding it
  }
  ~Lock() { pthread_mutex_unlock(m_); }

 private:
  pthread_mutex_t* m_;
};

class ShmStore {
 public:
  ShmStore(const std::string& name, uint64_t capacity, bool create, uint64_t table_cap)
      : name_(name), owner_(create) {
    if (create) {
      shm_unlink(name.c_str());
      fd_ = shm_open(name.c_str(), O_CREAT | O_RDWR | O_EXCL, 0600);
      if (fd_ < 0) throw std::runtime_error("shm_open(create) failed: " + std::string(strerror(errno)));
      uint64_t tbl_bytes = table_cap * sizeof(Entry);
      uint64_t hdr = (sizeof(Header) + kAlign - 1) / kAlign * kAlign;
      uint64_t arena_off = (hdr + tbl_bytes + kAlign - 1) / kAlign * kAlign;
      size_ = arena_off + (capacity + kAlign - 1) / kAlign * kAlign;
      if (ftruncate(fd_, (off_t)size_) != 0) throw std::runtime_error("ftruncate failed");
      map();
      Header* h = H();
      memset(h, 0, sizeof(Header));
      h->total_size = size_;
      h->table_offset = hdr;
      h->table_cap = table_cap;
      h->arena_offset = arena_off;
      h->arena_size = size_ - arena_off;
      memset(base_ + hdr, 0, tbl_bytes);
      pthread_mutexattr_t a;
      pthread_mutexattr_init(&a);
      pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
      pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
      pthread_mutex_init(&h->mu, &a);
      // one big free block
      Block* b = blk(0);
      b->size = h->arena_size;
      b->prev_size = 0;
      b->free = 1;
      b->next_free = kNone;
      b->prev_free = kNone;
      h->free_head = 0;
      __sync_synchronize();
      h->magic = kMagic;
    } else {
      fd_ = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("shm_open(attach) failed: " + std::string(strerror(errno)));
      struct stat st;
      fstat(fd_, &st);
      size_ = (uint64_t)st.st_size;
      map();
      if (H()->magic != kMagic) throw std::runtime_error("shm store not initialised");
    }
  }

  ~ShmStore() {
    if (base_) munmap(base_, size_);
    if (fd_ >= 0) close(fd_);
  }

  void unlink() { shm_unlink(name_.c_str()); }

  // returns payload offset, or -1 if out of memory, -2 if the id exists
  int64_t create(py::bytes id, uint64_t size) {
    std::string s = id;
    Lock l(&H()->mu);
    if (find(s) >= 0) return -2;
    uint64_t off = alloc(size);
    if (off == kNone) return -1;
    int64_t slot = insert_slot(s);
    if (slot < 0) {
      free_block(off);
      return -1;
    }
    Entry* e = tbl() + slot;
    memset(e->id, 0, kIdLen);
    memcpy(e->id, s.data(), s.size());
    e->id_len = (uint32_t)s.size();
    e->offset = H()->arena_offset + off + sizeof(Block);
    e->size = size;
    e->pins = 1;  // the creator holds a pin until seal
    e->lru = ++H()->lru_clock;
    e->delete_pending = 0;
    __sync_synchronize();
    e->state = CREATED;
    H()->num_objects++;
    H()->used_bytes += blk(off)->size;
    return (int64_t)e->offset;
  }

  bool seal(py::bytes id) {
    std::string s = id;
    Lock l(&H()->mu);
    int64_t i = find(s);
    if (i < 0) return false;
    Entry* e = tbl() + i;
    e->state = SEALED;
    e->pins -= 1;
    maybe_free(i);
    return true;
  }

  // abort an unsealed create
  bool abort(py::bytes id) {
    std::string s = id;
    Lock l(&H()->mu);
    int64_t i = find(s);
    if (i < 0) return false;
    Entry* e = tbl() + i;
    e->pins = 0;
    e->delete_pending = 1;
    maybe_free(i);
    return true;
  }

  // pin + return (offset, size) of a sealed object; (-1, 0) if absent/unsealed
  py::tuple get(py::bytes id) {
    std::string s = id;
    Lock l(&H()->mu);
    int64_t i = find(s);
    if (i < 0) return py::make_tuple(-1, 0);
    Entry* e = tbl() + i;
    if (e->state != SEALED || e->delete_pending) return py::make_tuple(-1, 0);
    e->pins += 1;
    e->lru = ++H()->lru_clock;
    return py::make_tuple((int64_t)e->offset, (int64_t)e->size);
  }

  bool contains(py::bytes id) {
    std::string s = id;
    Lock l(&H()->mu);
    int64_t i = find(s);
    return i >= 0 && tbl()[i].state == SEALED && !tbl()[i].delete_pending;
  }

  void release(py::bytes id) {
    std::string s = id;
    Lock l(&H()->mu);
    int64_t i = find(s);
    if (i < 0) return;
    Entry* e = tbl() + i;
    if (e->pins > 0) e->pins -= 1;
    maybe_free(i);
  }

  // delete: frees now if unpinned, else when the last pin is released. Returns true if the id existed.
  bool remove(py::bytes id) {
    std::string s = id;
    Lock l(&H()->mu);
    int64_t i = find(s);
    if (i < 0) return false;
    tbl()[i].delete_pending = 1;
    maybe_free(i);
    return true;
  }

  // up to n sealed, unpinned objects in LRU order (spill candidates): list of (id, size)
  py::list lru_candidates(int n) {
    std::vector<std::pair<uint64_t, int64_t>> c;
    {
      Lock l(&H()->mu);
      for (uint64_t i = 0; i < H()->table_cap; ++i) {
        Entry* e = tbl() + i;
        if (e->state == SEALED && e->pins == 0 && !e->delete_pending) c.push_back({e->lru, (int64_t)i});
      }
      std::sort(c.begin(), c.end());
      py::list out;
      for (int k = 0; k < (int)c.size() && k < n; ++k) {
        Entry* e = tbl() + c[k].second;
        out.append(py::make_tuple(py::bytes((const char*)e->id, e->id_len), (int64_t)e->size));
      }
      return out;
    }
  }

  py::dict stats() {
    Lock l(&H()->mu);
    py::dict d;
    d["capacity"] = H()->arena_size;
    d["used_bytes"] = H()->used_bytes;
    d["num_objects"] = H()->num_objects;
    uint64_t largest = 0, nfree = 0;
    for (uint64_t o = H()->free_head; o != kNone; o = blk(o)->next_free) {
      largest = std::max(largest, blk(o)->size);
      ++nfree;
    }
    d["largest_free"] = largest > sizeof(Block) ? largest - sizeof(Block) : 0;
    d["free_blocks"] = nfree;
    return d;
  }

  uint64_t address() const { return (uint64_t)base_; }
  uint64_t size() const { return size_; }
  std::string name() const { return name_; }

  // raw view helpers for Python (memoryview over [offset, offset+len))
  py::memoryview view(uint64_t offset, uint64_t len, bool readonly) {
    if (offset + len > size_) throw std::out_of_range("view out of range");
    return py::memoryview::from_memory(base_ + offset, (ssize_t)len, readonly);
  }

  void write(uint64_t offset, py::buffer b) {
    py::buffer_info info = b.request();
    uint64_t n = (uint64_t)info.size * info.itemsize;
    if (offset + n > size_) throw std::out_of_range("write out of range");
    py::gil_scoped_release rel;
    memcpy(base_ + offset, info.ptr, n);
  }

 private:
  void map() {
    void* p = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (p == MAP_FAILED) throw std::runtime_error("mmap failed");
    base_ = (uint8_t*)p;
  }
  Header* H() const { return (Header*)base_; }
  Entry* tbl() const { return (Entry*)(base_ + H()->table_offset); }
  Block* blk(uint64_t off) const { return (Block*)(base_ + H()->arena_offset + off); }

  int64_t find(const std::string& s) const {
    const uint64_t cap = H()->table_cap;
    uint64_t i = hash_id((const uint8_t*)s.data(), (int)s.size()) % cap;
    for (uint64_t n = 0; n < cap; ++n, i = (i + 1) % cap) {
      Entry* e = tbl() + i;
      if (e->state == EMPTY) return -1;
      if (e->state != TOMBSTONE && e->id_len == s.size() && memcmp(e->id, s.data(), s.size()) == 0) return (int64_t)i;
    }
    return -1;
  }

  int64_t insert_slot(const std::string& s) {
    if (s.size() > (size_t)kIdLen) return -1;
    const uint64_t cap = H()->table_cap;
    uint64_t i = hash_id((const uint8_t*)s.data(), (int)s.size()) % cap;
    for (uint64_t n = 0; n < cap; ++n, i = (i + 1) % cap) {
      Entry* e = tbl() + i;
      if (e->state == EMPTY || e->state == TOMBSTONE) {
        if (e->state == TOMBSTONE) H()->num_tombstones--;
        return (int64_t)i;
      }
    }
    return -1;
  }

  void maybe_free(int64_t i) {
    Entry* e = tbl() + i;
    if (!e->delete_pending || e->pins > 0) return;
    uint64_t off = e->offset - H()->arena_offset - sizeof(Block);
    H()->used_bytes -= blk(off)->size;
    free_block(off);
    e->state = TOMBSTONE;
    H()->num_tombstones++;
    H()->num_objects--;
    // rebuild runs of tombstones lazily: if the next slot is EMPTY, this slot can become EMPTY too
    const uint64_t cap = H()->table_cap;
    uint64_t j = i;
    while (tbl()[(j + 1) % cap].state == EMPTY && tbl()[j].state == TOMBSTONE) {
      tbl()[j].state = EMPTY;
      H()->num_tombstones--;
      j = (j + cap - 1) % cap;
    }
  }

  // ---------------------------------------------------------------- allocator
  void fl_remove(uint64_t o) {
    Block* b = blk(o);
    if (b->prev_free != kNone) blk(b->prev_free)->next_free = b->next_free; else H()->free_head = b->next_free;
    if (b->next_free != kNone) blk(b->next_free)->prev_free = b->prev_free;
    b->next_free = b->prev_free = kNone;
  }
  void fl_push(uint64_t o) {
    Block* b = blk(o);
    b->prev_free = kNone;
    b->next_free = H()->free_head;
    if (H()->free_head != kNone) blk(H()->free_head)->prev_free = o;
    H()->free_head = o;
  }

  uint64_t alloc(uint64_t payload) {
    uint64_t need = (payload + sizeof(Block) + kAlign - 1) / kAlign * kAlign;
    if (need < 2 * kAlign) need = 2 * kAlign;
    // first fit
    for (uint64_t o = H()->free_head; o != kNone; o = blk(o)->next_free) {
      Block* b = blk(o);
      if (b->size < need) continue;
      fl_remove(o);
      uint64_t rest = b->size - need;
      if (rest >= 2 * kAlign) {
        b->size = need;
        uint64_t no = o + need;
        Block* nb = blk(no);
        nb->size = rest;
        nb->prev_size = need;
        nb->free = 1;
        uint64_t after = no + rest;
        if (after < H()->arena_size) blk(after)->prev_size = rest;
        fl_push(no);
      }
      b->free = 0;
      return o;
    }
    return kNone;
  }

  void free_block(uint64_t o) {
    Block* b = blk(o);
    b->free = 1;
    // coalesce with next
    uint64_t next = o + b->size;
    if (next < H()->arena_size && blk(next)->free) {
      fl_remove(next);
      b->size += blk(next)->size;
    }
    // coalesce with previous
    if (o > 0) {
      uint64_t prev = o - b->prev_size;
      if (blk(prev)->free) {
        fl_remove(prev);
        blk(prev)->size += b->size;
        o = prev;
        b = blk(o);
      }
    }
    uint64_t after = o + b->size;
    if (after < H()->arena_size) blk(after)->prev_size = b->size;
    fl_push(o);
  }

  std::string name_;
  bool owner_;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  uint64_t size_ = 0;
};

// A pinned, read-only (or writable) window onto one object. Exposes the buffer protocol so
// memoryview/numpy/torch views alias shm directly; the pin is released when the last view dies.
struct PinnedView {
  py::object store_obj;  // keeps the mapping alive
  ShmStore* store;
  std::string id;
  uint64_t offset, len;
  bool readonly;
  bool released = false;
  ~PinnedView() {
    if (!released && store) {
      try {
        store->release(py::bytes(id));
      } catch (...) {
      }
    }
  }
};

// Large-object copy into the segment with several threads (reference: the Plasma client's
// `memcopy_threads` / src/ray/util/memory.cc parallel memcopy): one core's memcpy tops out well
// below the socket's bandwidth, and the first touch of fresh shm pages faults them in, which
// then also runs in parallel. Chunks are page aligned.
static void parallel_memcpy(uint8_t* dst, const uint8_t* src, size_t n, int threads) {
  constexpr size_t kMin = 8u << 20;
  if (threads <= 1 || n < kMin) {
    memcpy(dst, src, n);
    return;
  }
  threads = (int)std::min<size_t>((size_t)threads, n / (kMin / 4));
  const size_t chunk = ((n + threads - 1) / threads + 4095) & ~(size_t)4095;
  std::vector<std::thread> ts;
  for (int t = 1; t < threads; ++t) {
    const size_t off = chunk * t;
    if (off >= n) break;
    const size_t len = std::min(chunk, n - off);
    ts.emplace_back([=] { memcpy(dst + off, src + off, len); });
  }
  memcpy(dst, src, std::min(chunk, n));
  for (auto& th : ts) th.join();
}

void register_store(py::module_& m) {
  m.def(
      "copy_into",
      [](py::buffer dst, py::buffer src, int threads) {
        py::buffer_info di = dst.request(true), si = src.request();
        const size_t n = (size_t)si.size * si.itemsize;
        if (n > (size_t)di.size * di.itemsize) throw std::out_of_range("copy_into: destination too small");
        py::gil_scoped_release rel;
        parallel_memcpy((uint8_t*)di.ptr, (const uint8_t*)si.ptr, n, threads);
      },
      py::arg("dst"), py::arg("src"), py::arg("threads") = 4);
  py::class_<PinnedView>(m, "PinnedView", py::buffer_protocol())
      .def_buffer([](PinnedView& v) -> py::buffer_info {
        return py::buffer_info((void*)(v.store->address() + v.offset), 1, py::format_descriptor<uint8_t>::format(), 1,
                               {(ssize_t)v.len}, {(ssize_t)1}, v.readonly);
      })
      .def_readonly("offset", &PinnedView::offset)
      .def_readonly("length", &PinnedView::len)
      .def("__len__", [](const PinnedView& v) { return v.len; });
  m.def("pin_view", [](py::object store_obj, py::bytes id, bool readonly) -> py::object {
    ShmStore* st = store_obj.cast<ShmStore*>();
    py::tuple t = st->get(id);
    int64_t off = t[0].cast<int64_t>();
    if (off < 0) return py::none();
    auto* v = new PinnedView();
    v->store_obj = store_obj;
    v->store = st;
    v->id = id;
    v->offset = (uint64_t)off;
    v->len = (uint64_t)t[1].cast<int64_t>();
    v->readonly = readonly;
    return py::cast(v, py::return_value_policy::take_ownership);
  });
  py::class_<ShmStore>(m, "ShmStore")
      .def(py::init<const std::string&, uint64_t, bool, uint64_t>(), py::arg("name"), py::arg("capacity") = 0,
           py::arg("create") = false, py::arg("table_cap") = 1 << 18)
      .def("create", &ShmStore::create)
      .def("seal", &ShmStore::seal)
      .def("abort", &ShmStore::abort)
      .def("get", &ShmStore::get)
      .def("contains", &ShmStore::contains)
      .def("release", &ShmStore::release)
      .def("remove", &ShmStore::remove)
      .def("lru_candidates", &ShmStore::lru_candidates)
      .def("stats", &ShmStore::stats)
      .def("view", &ShmStore::view, py::arg("offset"), py::arg("length"), py::arg("readonly") = true)
      .def("write", &ShmStore::write)
      .def("unlink", &ShmStore::unlink)
      .def_property_readonly("address", &ShmStore::address)
      .def_property_readonly("size", &ShmStore::size)
      .def_property_readonly("name", &ShmStore::name);
}
