// ggrs_amd/csrc/wire.hip — batched input packets: the
// encode of UdpProtocol::send_pending_output (protocol.rs:468-500) and the
// decode of UdpProtocol::on_input (protocol.rs:616-689) for one endpoint per
// (session, remote handle), straight into the P2P batch's delivery tensors.
//
// Wire format (network/compression.rs): XOR delta of every pending input
// against the reference input (the last acked one), then bitfield RLE
// (bitfield-rle 0.2): varint-headed sequences, odd header = a run of
// `header >> 2` bytes of 0x00 / 0xFF (bit 1), even header = `header >> 1`
// literal bytes.  Varints are unsigned LEB128.  The encoder compresses runs of
// >= 4 equal 0x00/0xFF bytes (the same rule as oracle/ggrs_oracle.hpp wire::).
//
// One lane per endpoint: packets are a few bytes (one input per frame since
// the last ack), so the work is a short serial parse per lane; lanes of a wave
// read consecutive packet rows and write consecutive sessions of one frame.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ggrs_amd.h"

namespace {

constexpr int32_t kNull = -1;
constexpr int kRunMin = 4;

// status codes per endpoint (rb_decode_input_packets)
constexpr int32_t kDecOk = 0, kDecNothing = 1, kDecMalformed = -1, kDecGap = -2;

struct DecParams {
  const uint8_t* packets;
  int64_t packet_stride;
  const int32_t* lengths;
  const int32_t* start_frames;
  uint8_t* remote_inputs;  // [remote_frames][P][S] Input values of input_bytes
  int32_t* remote_upto;    // [P][S]
  int32_t* status;         // [S]
  int32_t handle, P, S, IB, remote_frames, max_prediction;
};

__device__ __forceinline__ uint8_t in_byte(const uint8_t* base, int32_t f, int h, int P, int S, int s, int IB, int i) {
  return base[((static_cast<size_t>(f) * P + h) * S + s) * IB + i];
}

__global__ void __launch_bounds__(256) decode_packets_kernel(const DecParams p) {
  const int s = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
  if (s >= p.S) return;
  const int h = p.handle, IB = p.IB;
  int32_t* up = p.remote_upto + static_cast<size_t>(h) * p.S + s;
  const int32_t last = *up;
  const int32_t start = p.start_frames[s];
  const int32_t n = p.lengths[s];
  const uint8_t* d = p.packets + static_cast<int64_t>(s) * p.packet_stride;
  if (n <= 0) {  // no packet from this endpoint this tick
    p.status[s] = kDecNothing;
    return;
  }
  // a length past the row would read the next endpoint's packet (or past the tensor): the
  // datagram is not what the row holds, so it is malformed
  if (n > p.packet_stride) {
    p.status[s] = kDecMalformed;
    return;
  }
  // protocol.rs:639-642: a packet must not skip frames we never received
  if (last != kNull && last + 1 < start) {
    p.status[s] = kDecGap;
    return;
  }
  // protocol.rs:646-653: decode against the input before start_frame (blank
  // before the first input); recv_inputs keeps only the last 2*max_prediction
  // frames, so an older reference means the packet is ignored
  if (last != kNull && start - 1 < last - 2 * p.max_prediction) {
    p.status[s] = kDecNothing;
    return;
  }
  // recv_inputs never holds a frame below NULL_FRAME: such a packet finds no
  // decode input and is ignored (protocol.rs:653); a reference input past the
  // caller's remote_inputs tensor cannot be read at all
  if (last != kNull && start - 1 < kNull) {
    p.status[s] = kDecNothing;
    return;
  }
  if (start - 1 >= p.remote_frames) {
    p.status[s] = kDecMalformed;
    return;
  }
  uint8_t ref[4] = {0, 0, 0, 0};  // recv_inputs[NULL_FRAME] is the zeroed input (protocol.rs:213-214)
  if (last != kNull && start - 1 != kNull)
    for (int i = 0; i < IB; ++i) ref[i] = in_byte(p.remote_inputs, start - 1, h, p.P, p.S, s, IB, i);
  // bitfield RLE decode fused with delta decode: byte k of the XOR stream is
  // byte (k % IB) of input k / IB
  int32_t k = 0, newest = last;
  uint8_t cur[4] = {0, 0, 0, 0};
  auto emit = [&](uint8_t x) {
    const int i = k % IB;
    cur[i] = static_cast<uint8_t>(ref[i] ^ x);
    if (i == IB - 1) {
      const int32_t f = start + k / IB;
      if (f > last && f < p.remote_frames) {  // protocol.rs:661-663: skip inputs already received
        uint8_t* dst = p.remote_inputs + ((static_cast<size_t>(f) * p.P + h) * p.S + s) * IB;
        for (int j = 0; j < IB; ++j) dst[j] = cur[j];
        newest = f;
      }
    }
    ++k;
  };
  int32_t pos = 0;
  bool ok = true;
  while (pos < n && ok) {
    uint32_t hdr = 0;
    int shift = 0;
    bool done = false;
    while (pos < n && shift < 35) {  // LEB128
      const uint8_t b = d[pos++];
      hdr |= static_cast<uint32_t>(b & 0x7F) << shift;
      shift += 7;
      if (!(b & 0x80)) {
        done = true;
        break;
      }
    }
    if (!done) {
      ok = false;
      break;
    }
    if (hdr & 1u) {  // compressed run of 0x00 / 0xFF
      const uint32_t len = hdr >> 2;
      if (len > (1u << 16)) {
        ok = false;
        break;
      }
      const uint8_t x = (hdr & 2u) ? 0xFF : 0x00;
      for (uint32_t i = 0; i < len; ++i) emit(x);
    } else {  // literal bytes
      const uint32_t len = hdr >> 1;
      if (len > static_cast<uint32_t>(n - pos)) {
        ok = false;
        break;
      }
      for (uint32_t i = 0; i < len; ++i) emit(d[pos++]);
    }
  }
  if (ok && k % IB != 0) ok = false;  // compression.rs:47 assert: whole inputs only
  if (!ok) {
    p.status[s] = kDecMalformed;  // the reference panics ("decoding failed", protocol.rs:656)
    return;
  }
  *up = newest;
  p.status[s] = newest == last ? kDecNothing : kDecOk;
}

struct EncParams {
  const uint8_t* inputs;  // [frames][P][S] Input values by frame (the sender's local inputs)
  int32_t frames;
  const int32_t* acked;   // [S] last frame the receiver acked (kNull: none)
  const int32_t* newest;  // [S] newest frame to send
  uint8_t* packets;
  int64_t packet_stride;
  int32_t* lengths;
  int32_t* start_frames;
  int32_t handle, P, S, IB, first_frame;
};

__device__ __forceinline__ void put_varint(uint8_t* out, int32_t cap, int32_t& pos, uint32_t v, bool& ok) {
  while (v >= 0x80) {
    if (pos >= cap) {
      ok = false;
      return;
    }
    out[pos++] = static_cast<uint8_t>(v | 0x80);
    v >>= 7;
  }
  if (pos >= cap) {
    ok = false;
    return;
  }
  out[pos++] = static_cast<uint8_t>(v);
}

// send_pending_output: pending inputs (acked, newest] XOR the last acked input
// (blank before any ack), bitfield-RLE encoded.
__global__ void __launch_bounds__(256) encode_packets_kernel(const EncParams p) {
  const int s = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
  if (s >= p.S) return;
  const int h = p.handle, IB = p.IB;
  const int32_t acked = p.acked[s], newest = p.newest[s];
  // pending_output starts after the last ack, or at the sender's first input
  // (its input delay) before any ack (protocol.rs:471-476)
  const int32_t start = acked == kNull ? p.first_frame : acked + 1;
  uint8_t* out = p.packets + static_cast<int64_t>(s) * p.packet_stride;
  const int32_t cap = static_cast<int32_t>(p.packet_stride);
  p.start_frames[s] = start;
  if (newest < start || newest >= p.frames || start < 0) {
    p.lengths[s] = 0;
    return;
  }
  uint8_t ref[4] = {0, 0, 0, 0};
  if (acked != kNull)
    for (int i = 0; i < IB; ++i) ref[i] = in_byte(p.inputs, acked, h, p.P, p.S, s, IB, i);
  const int32_t total = (newest - start + 1) * IB;  // XOR stream length
  auto xb = [&](int32_t k) -> uint8_t {
    return static_cast<uint8_t>(ref[k % IB] ^ in_byte(p.inputs, start + k / IB, h, p.P, p.S, s, IB, k % IB));
  };
  int32_t pos = 0, lit = 0, k = 0;
  bool ok = true;
  auto flush = [&](int32_t end) {
    if (end > lit) {
      put_varint(out, cap, pos, static_cast<uint32_t>(end - lit) << 1, ok);
      for (int32_t i = lit; i < end && ok; ++i) {
        if (pos >= cap) ok = false;
        else out[pos++] = xb(i);
      }
    }
  };
  while (k < total && ok) {
    const uint8_t b = xb(k);
    int32_t j = k;
    if (b == 0x00 || b == 0xFF)
      while (j < total && xb(j) == b) ++j;
    if (j - k >= kRunMin) {
      flush(k);
      put_varint(out, cap, pos, (static_cast<uint32_t>(j - k) << 2) | (b ? 2u : 0u) | 1u, ok);
      k = lit = j;
    } else {
      k = j > k ? j : k + 1;
    }
  }
  flush(total);
  p.lengths[s] = ok ? pos : -1;  // -1: the packet does not fit packet_stride
}

}  // namespace

extern "C" {

rb_status rb_decode_input_packets(int32_t device, void* stream, int32_t handle, int32_t num_players,
                                  int32_t num_sessions, int32_t input_bytes, int32_t max_prediction,
                                  const uint8_t* packets, int64_t packet_stride, const int32_t* lengths,
                                  const int32_t* start_frames, void* remote_inputs, int32_t remote_frames,
                                  int32_t* remote_upto, int32_t* status) {
  if (handle < 0 || handle >= num_players || num_players > 4 || num_sessions <= 0 ||
      (input_bytes != 1 && input_bytes != 2 && input_bytes != 4) || max_prediction <= 0)
    return RB_INVALID_REQUEST;
  if (hipSetDevice(device) != hipSuccess) return RB_DEVICE_ERROR;
  DecParams p{packets, packet_stride, lengths, start_frames, static_cast<uint8_t*>(remote_inputs), remote_upto,
              status, handle, num_players, num_sessions, input_bytes, remote_frames, max_prediction};
  hipLaunchKernelGGL(decode_packets_kernel, dim3((num_sessions + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), p);
  return hipGetLastError() == hipSuccess ? RB_OK : RB_DEVICE_ERROR;
}

rb_status rb_encode_input_packets(int32_t device, void* stream, int32_t handle, int32_t num_players,
                                  int32_t num_sessions, int32_t input_bytes, const void* inputs, int32_t frames,
                                  int32_t first_frame, const int32_t* acked, const int32_t* newest, uint8_t* packets,
                                  int64_t packet_stride, int32_t* lengths, int32_t* start_frames) {
  if (handle < 0 || handle >= num_players || num_players > 4 || num_sessions <= 0 ||
      (input_bytes != 1 && input_bytes != 2 && input_bytes != 4) || packet_stride <= 0)
    return RB_INVALID_REQUEST;
  if (hipSetDevice(device) != hipSuccess) return RB_DEVICE_ERROR;
  EncParams p{static_cast<const uint8_t*>(inputs), frames, acked, newest, packets, packet_stride, lengths,
              start_frames, handle, num_players, num_sessions, input_bytes, first_frame};
  hipLaunchKernelGGL(encode_packets_kernel, dim3((num_sessions + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), p);
  return hipGetLastError() == hipSuccess ? RB_OK : RB_DEVICE_ERROR;
}

}  // extern "C"
