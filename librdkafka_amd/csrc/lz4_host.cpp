// lz4_host.cpp -- placeholder until the LZ4F engine lands.
#include "lz4_engine.h"
namespace rdk {
int lz4f_compress_host(Ctx *, size_t, int, int, void **, size_t *) {
  return set_error(RDK_HIP_E_HIP, "lz4f compress: not built yet");
}
int lz4f_decompress_host(Ctx *, int, uint8_t *, size_t, void **, size_t *) {
  return set_error(RDK_HIP_E_HIP, "lz4f decompress: not built yet");
}
}  // namespace rdk
