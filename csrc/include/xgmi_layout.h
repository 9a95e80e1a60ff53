// Shared layout constants of the xGMI all-reduce workspace
// (csrc/kernels/xgmi.hip device side, csrc/runtime/xgmi.cpp host side).
#pragma once

namespace edl_xgmi {
constexpr int kMaxRanks = 8;     // one MI355X node
constexpr int kMaxBlocks = 256;  // workgroups per collective (one per CU at most)
constexpr int kFlagBytes = 2 * kMaxRanks * kMaxBlocks * 4;  // [phase][src rank][block] uint32
}  // namespace edl_xgmi
