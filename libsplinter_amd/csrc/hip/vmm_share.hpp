// vmm_share.hpp — an HBM arena other processes can attach, built from HIP virtual-memory chunks.
//
// hipIpcGetMemHandle / hipIpcOpenMemHandle on one hipMalloc allocation is the obvious way to
// expose an arena to other processes ("cross-process GPU sharing"), but on the
// MI355X hosts (dmabuf IPC only, HSA_ENABLE_IPC_MODE_LEGACY=0) the import of an allocation past
// ~2 GiB never returns: 1.95 GiB attached in 0.15 s, 3.04 GiB hung (dev/debug/ipc_open_debug.py,
// gpurun_out/r2_31).  A 100M-key arena is ~70 GiB.  So the owner builds the arena from physical
// chunks (hipMemCreate, SPLINTER_HBM_CHUNK_MB, default 1024) mapped back to back into one
// reserved virtual range -- the kernels see one flat arena as before -- and exports every chunk
// as a dmabuf file descriptor.  An attaching process fetches those descriptors from the owner over
// a UNIX socket (SCM_RIGHTS; no ptrace-style pidfd_getfd, which needs the importer to be the
// owner's ancestor on hosts with Yama), imports each chunk and maps them back to back into its
// own reserved range.
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <poll.h>
#include <string>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <mutex>
#include <thread>
#include <sys/mman.h>
#include <unistd.h>
#include <vector>

namespace spl {

class VmmArena {
 public:
  ~VmmArena() { release(); }

  // Owner: reserve, create, map and export ceil(bytes / chunk) chunks.
  int create(int device, size_t bytes, size_t chunk_bytes) {
    device_ = device;
    hipMemAllocationProp p = prop(device);
    size_t g = 0;
    if (hipMemGetAllocationGranularity(&g, &p, hipMemAllocationGranularityRecommended) != hipSuccess || !g)
      g = 2u << 20;
    chunk_ = (chunk_bytes + g - 1) / g * g;
    const size_t n = (bytes + chunk_ - 1) / chunk_;
    if (reserve(n) != 0) return -1;
    for (size_t i = 0; i < n; ++i) {
      hipMemGenericAllocationHandle_t h;
      if (hipMemCreate(&h, chunk_, &p, 0) != hipSuccess) return fail();
      handles_.push_back(h);
      if (hipMemMap((uint8_t*)va_ + i * chunk_, chunk_, 0, h, 0) != hipSuccess) return fail();
      ++mapped_;
      int fd = -1;
      if (hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0) != hipSuccess) return fail();
      fds_.push_back(fd);
    }
    return access();
  }

  // Importer: map the owner's exported chunks (descriptors are consumed).
  int import(int device, const std::vector<int>& fds, size_t chunk_bytes) {
    device_ = device;
    chunk_ = chunk_bytes;
    if (fds.empty() || reserve(fds.size()) != 0) return -1;
    for (size_t i = 0; i < fds.size(); ++i) {
      hipMemGenericAllocationHandle_t h;
      int fd = fds[i];
      // The HIP runtime in the process decides how the descriptor is passed: ROCm 7.2 takes the fd
      // value cast to a pointer (as CUDA does), older runtimes -- e.g. the ROCm 7.0 copy a torch
      // wheel loads first -- dereference a pointer to it (SPLINTER_VMM_FD_BY_PTR overrides).
      const hipError_t e = hipMemImportFromShareableHandle(
          &h, fd_by_pointer() ? (void*)&fd : (void*)(intptr_t)fd, hipMemHandleTypePosixFileDescriptor);
      fds_.push_back(fds[i]);  // kept: host_map() maps the same dmabuf on the CPU side
      if (e != hipSuccess) {
        for (size_t j = i + 1; j < fds.size(); ++j) close(fds[j]);
        return fail();
      }
      handles_.push_back(h);
      if (hipMemMap((uint8_t*)va_ + i * chunk_, chunk_, 0, h, 0) != hipSuccess) {
        for (size_t j = i + 1; j < fds.size(); ++j) close(fds[j]);
        return fail();
      }
      ++mapped_;
    }
    return access();
  }

  // Host (CPU) view of the whole range, zero-copy: each chunk's dmabuf descriptor mmap'ed back to
  // back, so a device address d maps to host_map() + (d - base()).  The amdgpu driver serves the
  // mapping through the PCIe BAR: uncached, ~2.4 us per dependent host read on MI355X
  // (profiles/r2_hbm_host_map.md).  nullptr when the driver refuses the mapping.
  void* host_map() {
    std::lock_guard<std::mutex> lk(host_mu_);
    if (host_ || host_failed_) return host_;
    host_failed_ = true;
    if (fds_.empty() || fds_.size() != handles_.size()) return nullptr;
    const size_t total = chunk_ * fds_.size();
    void* r = mmap(nullptr, total, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (r == MAP_FAILED) return nullptr;
    for (size_t i = 0; i < fds_.size(); ++i) {
      void* m = mmap((uint8_t*)r + i * chunk_, chunk_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fds_[i], 0);
      if (m == MAP_FAILED) {
        munmap(r, total);
        return nullptr;
      }
    }
    host_ = r;
    host_bytes_ = total;
    host_failed_ = false;
    return host_;
  }

  void release() {
    if (host_) munmap(host_, host_bytes_);
    host_ = nullptr;
    host_failed_ = false;
    stop_server();
    for (int fd : fds_) close(fd);
    fds_.clear();
    if (va_) {
      for (size_t i = 0; i < mapped_; ++i) (void)hipMemUnmap((uint8_t*)va_ + i * chunk_, chunk_);
      for (auto h : handles_) (void)hipMemRelease(h);
      (void)hipMemAddressFree(va_, reserved_);
    }
    handles_.clear();
    mapped_ = 0;
    va_ = nullptr;
  }

  void* base() const { return va_; }
  size_t chunk() const { return chunk_; }
  size_t chunks() const { return handles_.size(); }

  // ---------------------------------------------------- descriptor passing --
  // Abstract-namespace socket "\0<name>": serve every connecting process one copy of the chunk
  // descriptors (header {u64 n, u64 chunk}, then the fds in SCM_RIGHTS batches).  The chunk fds
  // map the whole arena read-write, so a peer gets them only if it could open the store's
  // descriptor itself: same uid (or root), or the descriptor file's group / other rw bits admit it
  // (SO_PEERCRED against the mode the store was created with, SPLINTER_DEFAULT_UMASK included).
  int serve(const std::string& name, const std::string& desc_path = std::string()) {
    sock_ = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (sock_ < 0) return -1;
    sockaddr_un a;
    socklen_t len = addr(name, &a);
    if (bind(sock_, (sockaddr*)&a, len) != 0 || listen(sock_, 16) != 0) {
      close(sock_);
      sock_ = -1;
      return -1;
    }
    stop_ = false;
    server_ = std::thread([this, desc_path] {
      while (!stop_.load()) {
        pollfd pf{sock_, POLLIN, 0};
        if (::poll(&pf, 1, 100) <= 0) continue;
        int c = accept4(sock_, nullptr, nullptr, SOCK_CLOEXEC);
        if (c < 0) continue;
        if (peer_allowed(c, desc_path)) send_fds(c);
        close(c);
      }
    });
    return 0;
  }

  // Importer side: connect to the owner's socket and receive the chunk descriptors.
  static int fetch(const std::string& name, std::vector<int>* fds, size_t* chunk) {
    int c = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (c < 0) return -1;
    sockaddr_un a;
    socklen_t len = addr(name, &a);
    if (connect(c, (sockaddr*)&a, len) != 0) {
      close(c);
      return -1;
    }
    uint64_t hdr[2] = {0, 0};
    int rc = -1;
    size_t got = 0;
    for (;;) {
      uint8_t buf[16];
      char ctl[CMSG_SPACE(sizeof(int) * kBatch)];
      iovec iov{buf, got == 0 && fds->empty() ? sizeof hdr : 1};
      msghdr m{};
      m.msg_iov = &iov;
      m.msg_iovlen = 1;
      m.msg_control = ctl;
      m.msg_controllen = sizeof ctl;
      const ssize_t r = recvmsg(c, &m, MSG_CMSG_CLOEXEC);
      if (r <= 0) break;
      if (fds->empty() && got == 0) {
        std::memcpy(hdr, buf, sizeof hdr);
        got = 1;
      }
      for (cmsghdr* cm = CMSG_FIRSTHDR(&m); cm; cm = CMSG_NXTHDR(&m, cm))
        if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) {
          const size_t k = (cm->cmsg_len - CMSG_LEN(0)) / sizeof(int);
          const int* p = (const int*)CMSG_DATA(cm);
          for (size_t i = 0; i < k; ++i) fds->push_back(p[i]);
        }
      if (hdr[0] && fds->size() >= hdr[0]) { rc = 0; break; }
    }
    close(c);
    if (rc == 0) *chunk = hdr[1];
    else {
      for (int fd : *fds) close(fd);
      fds->clear();
    }
    return rc;
  }

 private:
  static constexpr size_t kBatch = 64;

  static bool peer_allowed(int c, const std::string& desc_path) {
    ucred cr{};
    socklen_t cl = sizeof cr;
    if (getsockopt(c, SOL_SOCKET, SO_PEERCRED, &cr, &cl) != 0) return false;
    if (cr.uid == 0 || cr.uid == geteuid()) return true;
    struct stat st;
    if (desc_path.empty() || stat(desc_path.c_str(), &st) != 0) return false;
    if ((st.st_mode & 0006) == 0006) return true;                       // world read-write
    return (st.st_mode & 0060) == 0060 && cr.gid == st.st_gid;          // group read-write
  }

  static bool fd_by_pointer() {
    if (const char* e = getenv("SPLINTER_VMM_FD_BY_PTR")) return atoi(e) != 0;
    int v = 0;
    (void)hipRuntimeGetVersion(&v);
    return v < 70200000;  // HIP_VERSION = major * 1e7 + minor * 1e5 + patch
  }

  static hipMemAllocationProp prop(int device) {
    hipMemAllocationProp p;
    std::memset(&p, 0, sizeof p);
    p.type = hipMemAllocationTypePinned;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = device;
    return p;
  }
  static socklen_t addr(const std::string& name, sockaddr_un* a) {
    std::memset(a, 0, sizeof *a);
    a->sun_family = AF_UNIX;
    const size_t n = std::min(name.size(), sizeof(a->sun_path) - 2);
    std::memcpy(a->sun_path + 1, name.data(), n);  // abstract namespace: leading NUL
    return (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
  }
  void* host_ = nullptr;
  size_t host_bytes_ = 0;
  bool host_failed_ = false;
  std::mutex host_mu_;

  int reserve(size_t n) {
    reserved_ = n * chunk_;
    if (hipMemAddressReserve(&va_, reserved_, chunk_, nullptr, 0) != hipSuccess) {
      va_ = nullptr;
      return -1;
    }
    return 0;
  }
  int access() {
    hipMemAccessDesc d;
    std::memset(&d, 0, sizeof d);
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = device_;
    d.flags = hipMemAccessFlagsProtReadWrite;
    return hipMemSetAccess(va_, mapped_ * chunk_, &d, 1) == hipSuccess ? 0 : fail();
  }
  int fail() {
    release();
    return -1;
  }
  void send_fds(int c) {
    const uint64_t hdr[2] = {fds_.size(), chunk_};
    for (size_t off = 0; off < fds_.size() || off == 0; off += kBatch) {
      const size_t k = std::min(kBatch, fds_.size() - off);
      char ctl[CMSG_SPACE(sizeof(int) * kBatch)];
      std::memset(ctl, 0, sizeof ctl);
      uint8_t one = 0;
      iovec iov{off == 0 ? (void*)hdr : (void*)&one, off == 0 ? sizeof hdr : 1};
      msghdr m{};
      m.msg_iov = &iov;
      m.msg_iovlen = 1;
      m.msg_control = ctl;
      m.msg_controllen = CMSG_SPACE(sizeof(int) * k);
      cmsghdr* cm = CMSG_FIRSTHDR(&m);
      cm->cmsg_level = SOL_SOCKET;
      cm->cmsg_type = SCM_RIGHTS;
      cm->cmsg_len = CMSG_LEN(sizeof(int) * k);
      std::memcpy(CMSG_DATA(cm), fds_.data() + off, sizeof(int) * k);
      if (sendmsg(c, &m, MSG_NOSIGNAL) < 0) return;
      if (fds_.empty()) return;
    }
  }
  void stop_server() {
    if (server_.joinable()) {
      stop_ = true;
      server_.join();
    }
    if (sock_ >= 0) close(sock_);
    sock_ = -1;
  }

  int device_ = 0;
  void* va_ = nullptr;
  size_t reserved_ = 0, chunk_ = 0, mapped_ = 0;
  std::vector<hipMemGenericAllocationHandle_t> handles_;
  std::vector<int> fds_;
  int sock_ = -1;
  std::thread server_;
  std::atomic<bool> stop_{false};
};

}  // namespace spl
