// mck_internal.h -- engine-internal entry points shared between the
// engine's translation units (not part of the public C ABI).
#pragma once

extern "C" {
// Set this thread's mck_last_error() message ("" clears it).
void mck_internal_set_error(const char* msg);
}
