// Host-side native runtime of harp_amd (C ABI, loaded with ctypes).
#pragma once
#include <stddef.h>
#include <stdint.h>

#define HARP_HOST_EXPORT extern "C" __attribute__((visibility("default")))
