// cairo_amd/csrc/bitstream.cpp -- evx::bit_stream (reference bitstream.cpp),
// LSB-first bit container with bit indices and byte capacity.
#include "../../include/bitstream.h"

#include <cstring>
#include <new>

#include "../../include/cairo_amd.h"

namespace evx {

namespace {
inline uint32 bytes_for_bits(uint32 bits) { return (bits + 7) >> 3; }

// Copy count bits from src (starting at bit so) to dst (starting at bit dof),
// LSB-first, leaving the other bits of dst untouched.
void copy_bits(const uint8 *src, uint32 so, uint32 count, uint8 *dst, uint32 dof) {
  if (((so | dof) & 7) == 0) {
    memcpy(dst + (dof >> 3), src + (so >> 3), count >> 3);
    const uint32 done = count & ~7u;
    so += done;
    dof += done;
    count -= done;
  }
  while (count) {
    const uint32 sb = so & 7, db = dof & 7;
    uint32 n = 8 - (sb > db ? sb : db);
    if (n > count) n = count;
    const uint32 m = (1u << n) - 1u;
    const uint32 v = (src[so >> 3] >> sb) & m;
    uint8 &d = dst[dof >> 3];
    d = (uint8)((d & ~(m << db)) | (v << db));
    so += n;
    dof += n;
    count -= n;
  }
}
}  // namespace

bit_stream::bit_stream() : read_index(0), write_index(0), data_capacity(0), data_store(nullptr) {}

bit_stream::bit_stream(uint32 size_in_bits)
    : read_index(0), write_index(0), data_capacity(0), data_store(nullptr) {
  resize_capacity(size_in_bits);
}

bit_stream::bit_stream(void *bytes, uint32 size_in_bytes)
    : read_index(0), write_index(0), data_capacity(0), data_store(nullptr) {
  assign(bytes, size_in_bytes);
}

bit_stream::~bit_stream() { clear(); }

uint8 *bit_stream::query_data() const { return data_store; }
uint32 bit_stream::query_capacity() const { return data_capacity << 3; }
uint32 bit_stream::query_occupancy() const { return write_index - read_index; }
uint32 bit_stream::query_byte_occupancy() const { return bytes_for_bits(query_occupancy()); }

uint32 bit_stream::resize_capacity(uint32 size_in_bits) {
  if (!size_in_bits) return 0;
  clear();
  const uint32 n = bytes_for_bits(size_in_bits);
  data_store = new (std::nothrow) uint8[n];
  if (!data_store) return 0;
  memset(data_store, 0, n);
  data_capacity = n;
  return size_in_bits;
}

evx_status bit_stream::assign(void *bytes, uint32 size) {
  if (!bytes || !size) return EVX_ERROR_INVALIDARG;
  clear();
  data_store = new (std::nothrow) uint8[size];
  if (!data_store) return EVX_ERROR_OUTOFMEMORY;
  memcpy(data_store, bytes, size);
  read_index = 0;
  write_index = size << 3;
  data_capacity = size;
  return EVX_SUCCESS;
}

// Reference behaviour (bitstream.cpp:97-105): a seek past the end clamps the
// read index to the write index and still adds the offset.
void bit_stream::seek(uint32 offset) {
  if (read_index + offset >= write_index) read_index = write_index;
  read_index += offset;
}

void bit_stream::clear() {
  empty();
  delete[] data_store;
  data_store = nullptr;
  data_capacity = 0;
}

void bit_stream::empty() {
  write_index = 0;
  read_index = 0;
}

bool bit_stream::is_empty() const { return write_index == read_index; }
bool bit_stream::is_full() const { return write_index == query_capacity(); }

evx_status bit_stream::write_bit(uint8 value) {
  if (write_index + 1 > query_capacity()) return EVX_ERROR_CAPACITY_LIMIT;
  uint8 &d = data_store[write_index >> 3];
  const uint32 s = write_index & 7;
  d = (uint8)((d & ~(1u << s)) | ((value & 1u) << s));
  write_index++;
  return EVX_SUCCESS;
}

evx_status bit_stream::write_byte(uint8 value) { return write_bits(&value, 8); }

evx_status bit_stream::write_bits(void *data, uint32 count) {
  if (!data || !count) return EVX_ERROR_INVALIDARG;
  if (write_index + count > query_capacity()) return EVX_ERROR_CAPACITY_LIMIT;
  copy_bits((const uint8 *)data, 0, count, data_store, write_index);
  write_index += count;
  return EVX_SUCCESS;
}

evx_status bit_stream::write_bytes(void *data, uint32 count) { return write_bits(data, count << 3); }

evx_status bit_stream::peek_bit(void *data) {
  if (!data) return EVX_ERROR_INVALIDARG;
  if (read_index >= write_index) return EVX_ERROR_INVALID_RESOURCE;
  uint8 *d = (uint8 *)data;
  *d = (uint8)((*d & 0xFE) | ((data_store[read_index >> 3] >> (read_index & 7)) & 1u));
  return EVX_SUCCESS;
}

evx_status bit_stream::peek_bits(void *data, uint32 count) {
  if (!data || !count) return EVX_ERROR_INVALIDARG;
  if (read_index + count > write_index) return EVX_ERROR_INVALID_RESOURCE;
  copy_bits(data_store, read_index, count, (uint8 *)data, 0);
  return EVX_SUCCESS;
}

evx_status bit_stream::peek_byte(void *data) {
  if (!data) return EVX_ERROR_INVALIDARG;
  if (read_index + 8 > write_index) return EVX_ERROR_INVALID_RESOURCE;
  return peek_bits(data, 8);
}

evx_status bit_stream::peek_bytes(void *data, uint32 count) { return peek_bits(data, count << 3); }

evx_status bit_stream::read_bit(void *data) {
  const evx_status r = peek_bit(data);
  if (r == EVX_SUCCESS) read_index++;
  return r;
}

evx_status bit_stream::read_byte(void *data) {
  const evx_status r = peek_byte(data);
  if (r == EVX_SUCCESS) read_index += 8;
  return r;
}

evx_status bit_stream::read_bits(void *data, uint32 count) {
  const evx_status r = peek_bits(data, count);
  if (r == EVX_SUCCESS) read_index += count;
  return r;
}

evx_status bit_stream::read_bytes(void *data, uint32 count) { return read_bits(data, count << 3); }

}  // namespace evx

extern "C" {
void *evx_bitstream_create(uint32_t size_in_bits) {
  evx::bit_stream *b = new (std::nothrow) evx::bit_stream(size_in_bits);
  return b;
}
void evx_bitstream_destroy(void *bs) { delete (evx::bit_stream *)bs; }
const uint8_t *evx_bitstream_data(void *bs) { return ((evx::bit_stream *)bs)->query_data(); }
uint32_t evx_bitstream_occupancy(void *bs) { return ((evx::bit_stream *)bs)->query_occupancy(); }
void evx_bitstream_empty(void *bs) { ((evx::bit_stream *)bs)->empty(); }
int evx_bitstream_write_bits(void *bs, const void *data, uint32_t count) {
  return ((evx::bit_stream *)bs)->write_bits(const_cast<void *>(data), count);
}
}
