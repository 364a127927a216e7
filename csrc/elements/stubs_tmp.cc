// Temporary registration stubs (filled in by later milestones).
#include "decoders/decoders.h"
#include "elements/elements.h"

namespace nnsx {
void register_serial_decoders() {}
}  // namespace nnsx
