// Shared layout of the statevector "plan blob" consumed by the gfx950 pass kernels.
//
// A lowered circuit (Circuit.to_program: per gate kind,q0,q1,slot + scale,offset) is turned by the
// host planner (planner.cpp) into PASSES.  One pass = one kernel launch that streams every tile of
// every sample's state once: a tile is 2^k amplitudes whose index bits are k chosen qubits
// ("tile qubits"), held as R amplitudes per thread in registers (RB = log2 R "register bits") and
// TB = k - RB "thread bits".  Inside a pass, gates on register bits are pure VALU; gates on other
// tile qubits are reached by REMAP micro-ops: one LDS round trip that re-assigns which tile bits
// live in registers and, in the same trip, applies the pending GF(2)-linear permutation of fused
// CNOT chains.  Diagonal gates (RZ/P/Z/S/T/CZ) act on any bit, even qubits outside the tile.
#pragma once
// (no <stdint.h>: this header is also compiled by hiprtc)

namespace qfx {

// gate kinds (quantum/circuit.py KIND)
enum Kind : int {
  K_RX = 0, K_RY = 1, K_RZ = 2, K_P = 3, K_H = 4, K_X = 5, K_Y = 6, K_Z = 7, K_S = 8, K_SDG = 9,
  K_T = 10, K_TDG = 11, K_SX = 12, K_CX = 13, K_CZ = 14, K_SWAP = 15,
  // stochastic Pauli (noise trajectories): the slot value selects I/X/Y/Z (0..3) per sample
  K_PAULI = 18
};

// micro-op codes (planner-internal U1/D1 are lowered to G1 groups / D1T before serialisation)
enum OpCode : int { OP_G1 = 1, OP_D1T = 2, OP_CX = 3, OP_CZ = 4, OP_REMAP = 5, OP_U1 = 6, OP_D1 = 7 };
constexpr int MAX_GROUP = 8;   // single-qubit gates fused into one register-bit group

// pass init / final modes
enum InitMode : int { INIT_LOAD = 0, INIT_PRODUCT = 1, INIT_PSI_LAMBDA = 2, INIT_LOAD_BOTH = 3 };
enum FinalFlag : int { FIN_STORE = 1, FIN_READOUT = 2 };

// physical bit encoding in micro-op operands:
//   p <  RB          register bit p
//   RB <= p < 32     thread bit p - RB
//   p >= 64          qubit (p - 64) outside the tile: its value is uniform per tile
constexpr int PHYS_NONTILE = 64;

// pass descriptor (int32 words at blob[pass_offset + field])
enum PassField : int {
  PF_K = 0, PF_TB = 1, PF_INIT = 2, PF_FINAL = 3, PF_NOPS = 4, PF_OPS = 5, PF_LAYOUT0 = 6,
  PF_NGRAD = 7, PF_NNONTILE = 8, PF_NREAD = 9, PF_FINAL_LAYOUT = 10,
  PF_TILEQ = 16,        // [24] tile qubits: tile bit j <-> qubit
  PF_NONTILE = 40,      // [32] non-tile qubits (ascending)
  PF_READ_PHYS = 72,    // [8]  readout qubit -> phys bit in the FINAL layout
  PF_LAM_PHYS = 80,     // [8]  readout qubit -> phys bit in the INITIAL layout (adjoint lambda init)
  PF_Q0 = 96,           // [24] phys bit -> qubit in the initial layout (product-state init)
  PF_GREG0 = 120,       // [32] initial layout: global amplitude offset of register r
  PF_GTHR0 = 152,       // [16] initial layout: global offset contributed by thread bit j
  PF_GREGF = 168,       // [32] final layout: global offset of register r
  PF_GTHRF = 200,       // [16] final layout: global offset of thread bit j
  PF_SIZE = 224
};

// blob header: [0]=n_qubits [1]=n_passes [2]=n_gates [3]=gate table offset [4]=prefix offset
// [5]=R [6]=n_readout [7]=n_theta  [8..8+n_passes) pass offsets
enum HeaderField : int {
  HF_N = 0, HF_NPASS = 1, HF_NGATES = 2, HF_GATES = 3, HF_PREFIX = 4, HF_R = 5, HF_NREAD = 6,
  HF_NTHETA = 7, HF_PASSES = 8
};

// gate table entry: 6 words: kind, q0, q1, slot, scale(f32 bits), offset(f32 bits)
constexpr int GATE_WORDS = 6;
// micro-op: 4 words: code, a, b, c
//   G1:    a = register bit, b = gate count, c = word offset of the gate-index list (execution
//          order; forward multiplies the 2x2s, adjoint applies inverses + gradients in list order)
//   D1T:   a = phys bit (thread bit or non-tile qubit), c = gate index (diagonal 1q gate)
//   CX:    a = control phys bit, b = target register bit, c = gate index
//   CZ:    a, b = phys bits, c = gate index
//   REMAP: a = word offset of the remap table [wr R][wt TB][rr R][rt TB]: LDS slot of register r /
//          thread bit j on write (GF(2) map and XOR swizzle already applied - both are linear) and
//          on read (new layout); slot(r, tl) = tab_r[r] ^ XOR_{j: bit j of tl} tab_t[j]
//          b = word offset of the new layout (phys -> tile bit; bookkeeping only)
constexpr int OP_WORDS = 4;

}  // namespace qfx
