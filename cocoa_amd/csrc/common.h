// Shared host-side helpers for libcocoa_hip.so.
#pragma once
#include <stdexcept>
#include <string>

namespace cocoa {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

}  // namespace cocoa

// last error for calls made without a context (host data layer, create)
void cocoa_set_global_error(const std::string& msg);
