/*
 * include/bitstream.h -- evx::bit_stream, the byte container of the EVX-1 API
 * (reference bitstream.h:43-92), restated for libcairo_amd.so.
 *
 * Layout is the reference's (vptr, read_index, write_index, data_capacity,
 * data_store: 32 bytes on LP64).  Bits are LSB-first within each byte;
 * indices count bits; capacity is kept in bytes.  empty() rewinds both
 * indices but keeps the stored bytes.  Writes beyond capacity fail with
 * EVX_ERROR_CAPACITY_LIMIT and write nothing.
 */
#ifndef CAIRO_BITSTREAM_H
#define CAIRO_BITSTREAM_H

#include "evx_base.h"

namespace evx {

class bit_stream {
  uint32 read_index;
  uint32 write_index;
  uint32 data_capacity;
  uint8 *data_store;

 public:
  bit_stream();
  bit_stream(uint32 size_in_bits);
  bit_stream(void *bytes, uint32 size_in_bytes);
  virtual ~bit_stream();

  uint8 *query_data() const;
  uint32 query_capacity() const;       /* bits */
  uint32 query_occupancy() const;      /* bits */
  uint32 query_byte_occupancy() const; /* bytes, rounded up */
  uint32 resize_capacity(uint32 size_in_bits);

  evx_status assign(void *bytes, uint32 size_in_bytes);

  void seek(uint32 offset);
  void clear();
  void empty();

  bool is_empty() const;
  bool is_full() const;

  evx_status write_byte(uint8 value);
  evx_status write_bit(uint8 value);
  evx_status write_bytes(void *data, uint32 count);
  evx_status write_bits(void *data, uint32 count);

  evx_status read_byte(void *data);
  evx_status read_bit(void *data);
  evx_status read_bytes(void *data, uint32 count);
  evx_status read_bits(void *data, uint32 count);

  evx_status peek_byte(void *data);
  evx_status peek_bit(void *data);
  evx_status peek_bytes(void *data, uint32 count);
  evx_status peek_bits(void *data, uint32 count);

  /* libcairo_amd extension (non-virtual, layout unchanged): direct access to
   * the tail so the entropy stage can append without per-bit calls. */
  uint32 query_write_index() const { return write_index; }
  void advance_write_index(uint32 bits) { write_index += bits; }
  uint32 query_read_index() const { return read_index; }
  void set_read_index(uint32 bits) { read_index = bits; }

 private:
  bit_stream(const bit_stream &);
  bit_stream &operator=(const bit_stream &);
};

}  // namespace evx

#endif
