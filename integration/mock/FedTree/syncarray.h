// Minimal stand-in for FedTree's SyncArray (syncarray.h) -- enough for the
// shim's compile/run test; NOT the reference file.
#pragma once
#include <vector>
#include <cstddef>
template <typename T> class SyncArray {
public:
    explicit SyncArray(size_t n = 0) : v_(n) {}
    size_t size() const { return v_.size(); }
    T *host_data() { return v_.data(); }
private:
    std::vector<T> v_;
};
