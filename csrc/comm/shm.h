// Named POSIX shared-memory blocks for same-host, multi-process hand-off of
// host tensors (edgesink / edgesrc connect-type=SHM, videotestsrc pool-shm).
//
// The reference's tensor_demux hands every branch a reference to the same
// buffer (gsttensor_demux.c:469-556) inside one process.  With one process per
// GPU the branches live in other processes: a producer allocates its frame
// ring in a named segment, the consumer process maps the same segment and --
// when it has a GPU -- registers the mapping with hipHostRegister, so each
// consumer DMAs its share over ITS OWN GPU's host link instead of every byte
// funnelling through the producer's GPU.
#pragma once

#include <cstddef>
#include <memory>
#include <string>

#include "runtime/memory.h"

namespace nnsx {
namespace comm {

class ShmSegment : public std::enable_shared_from_this<ShmSegment> {
 public:
  // the owner: shm_open(O_CREAT | O_EXCL) + ftruncate + mmap; the name is
  // unlinked when the owner's segment goes (mappings of peers stay valid)
  static std::shared_ptr<ShmSegment> create(const std::string& name, size_t bytes, std::string* err);
  // a peer: map an existing segment (cached per name in this process)
  static std::shared_ptr<ShmSegment> open(const std::string& name, size_t bytes, std::string* err);
  // the segment of this process holding [p, p + n) (nullptr: none) and p's offset in it
  static std::shared_ptr<ShmSegment> find(const void* p, size_t n, size_t* off);
  ~ShmSegment();

  char* base() const { return base_; }
  size_t size() const { return size_; }
  const std::string& name() const { return name_; }
  // hipHostRegister'ed: DMA reads / writes it at the pinned rate
  bool registered() const { return registered_; }
  // a Memory over [off, off + n) that keeps the segment mapped (PINNED when
  // registered, else HOST); its allocation() is the segment, so runs of
  // adjacent views go up as one DMA
  MemoryPtr view(size_t off, size_t n, Memory::Release release = nullptr);

 private:
  ShmSegment() = default;
  bool map(int fd, size_t bytes, std::string* err);
  std::string name_;
  char* base_ = nullptr;
  size_t size_ = 0;
  bool owner_ = false, registered_ = false;
  int dev_ = -1;
};

}  // namespace comm
}  // namespace nnsx
