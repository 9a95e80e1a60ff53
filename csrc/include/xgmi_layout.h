// Shared layout constants of the xGMI collective engine
// (csrc/kernels/xgmi.hip device side, csrc/runtime/xgmi.cpp host side).
#pragma once

namespace edl_xgmi {
constexpr int kMaxRanks = 8;     // one MI355X node
constexpr int kMaxBlocks = 256;  // workgroups per collective (one per CU at most)
constexpr int kPhases = 3;       // entry / after reduce-scatter / exit
constexpr int kFlagBytes = kPhases * kMaxRanks * kMaxBlocks * 4;  // [phase][src rank][block] uint32
// Host-mapped status record written by the first workgroup that gives up:
//   [0] 0 = healthy, 1 = a barrier gave up      [1] round      [2] phase
//   [3] workgroup index                          [4] missing peer rank
//   [5] flag value last seen from that peer      [6] waited (ms)
//   [7] reason: 1 = abort word, 2 = deadline
constexpr int kStatusWords = 8;
}  // namespace edl_xgmi
