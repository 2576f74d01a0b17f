/*
 * include/evx_base.h -- integer typedefs and evx_status codes of the EVX-1 API
 * (reference base.h:110-172), restated for the drop-in headers.
 */
#ifndef CAIRO_EVX_BASE_H
#define CAIRO_EVX_BASE_H

#include <stdint.h>

namespace evx {

typedef int64_t int64;
typedef int32_t int32;
typedef int16_t int16;
typedef int8_t int8;
typedef uint64_t uint64;
typedef uint32_t uint32;
typedef uint16_t uint16;
typedef uint8_t uint8;
typedef float float32;
typedef double float64;

typedef uint8 evx_status;

}  // namespace evx

#define EVX_SUCCESS (0)
#define EVX_ERROR_INVALIDARG (1)
#define EVX_ERROR_NOTIMPL (2)
#define EVX_ERROR_OUTOFMEMORY (3)
#define EVX_ERROR_UNDEFINED (4)
#define EVX_ERROR_HARDWAREFAIL (5)
#define EVX_ERROR_INVALID_INDEX (6)
#define EVX_ERROR_CAPACITY_LIMIT (7)
#define EVX_ERROR_INVALID_RESOURCE (8)
#define EVX_ERROR_OPERATION_TIMEDOUT (9)
#define EVX_ERROR_EXECUTION_FAILURE (10)
#define EVX_ERROR_PERMISSION_DENIED (11)
#define EVX_ERROR_IO_FAILURE (12)
#define EVX_ERROR_RESOURCE_UNREACHABLE (13)
#define EVX_ERROR_SYSTEM_FAILURE (14)
#define EVX_ERROR_NOT_READY (15)
#define EVX_ERROR_OPERATION_COMPLETED (16)
#define EVX_ERROR_RESOURCE_UNUSED (17)

#define evx_succeeded(status) ((status) == EVX_SUCCESS)
#define evx_failed(status) (!evx_succeeded(status))

#endif
