// cairo_amd/csrc/decoder.cpp -- evx1_decoder entry points (reference
// evx1dec.cpp, evx1.cpp:28-81).  The GPU decoder is a later milestone
// (SURVEY.md §8(f) F3); until then create_decoder reports EVX_ERROR_NOTIMPL.
#include "../../include/evx1.h"

namespace evx {

evx_status create_decoder(evx1_decoder **output) {
  if (!output) return EVX_ERROR_INVALIDARG;
  *output = nullptr;
  return EVX_ERROR_NOTIMPL;
}

evx_status destroy_decoder(evx1_decoder *input) {
  if (!input) return EVX_ERROR_INVALIDARG;
  return EVX_ERROR_NOTIMPL;
}

}  // namespace evx
