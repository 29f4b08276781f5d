-- lz4ada-gpu.ads -- bulk entry points of the GPU hot path (no reference
-- twin: SURVEY 8b "a per-block Update cannot reach the roofline").
-- A caller such as tool_unlz4ada can replace its Update loop for a whole
-- frame by one Decode_Frame call.  UNTESTED (no GNAT in this image).
with Interfaces;
with System;

package LZ4Ada.GPU is

	-- include/lz4ada_hip.h: lz4ada_decode_frame.  Raises the reference
	-- exception with the reference message on failure.
	procedure Decode_Frame(Frame:          in     Octets;
				Output:         in out Octets;
				Output_Length:  out    Interfaces.Integer_64;
				Frame_Consumed: out    Interfaces.Integer_64);

	-- lz4ada_decode_stream: every frame of a concatenated stream.
	procedure Decode_Stream(Input:         in     Octets;
				Output:        in out Octets;
				Output_Length: out    Interfaces.Integer_64);

	-- lz4ada_decoded_bound: output capacity needed by Decode_Stream.
	function Decoded_Bound(Input: in Octets) return Interfaces.Integer_64;

	-- lz4ada_decode_frame_multi: Decode_Frame over GPUs 0 .. N_GPUs-1 of
	-- this process (one host thread per device, RCCL for the verdict);
	-- frames that do not shard decode on GPU 0.  Same exceptions.
	procedure Decode_Frame_Multi(Frame:          in     Octets;
				N_GPUs:         in     Positive;
				Output:         in out Octets;
				Output_Length:  out    Interfaces.Integer_64;
				Frame_Consumed: out    Interfaces.Integer_64);

	-- lz4ada_rccl_version: the RCCL this process bound (22606 = 2.26.6).
	function RCCL_Version return Interfaces.Integer_32;
	pragma Import(C, RCCL_Version, "lz4ada_rccl_version");

private

	function C_Decode_Frame(Frame: System.Address; Len: Interfaces.Integer_64;
			Out_Buf: System.Address; Out_Cap: Interfaces.Integer_64;
			Out_Len, Consumed: access Interfaces.Integer_64)
			return Interfaces.Integer_32;
	pragma Import(C, C_Decode_Frame, "lz4ada_decode_frame");

	function C_Decode_Stream(Input: System.Address; Len: Interfaces.Integer_64;
			Out_Buf: System.Address; Out_Cap: Interfaces.Integer_64;
			Out_Len: access Interfaces.Integer_64)
			return Interfaces.Integer_32;
	pragma Import(C, C_Decode_Stream, "lz4ada_decode_stream");

	function C_Decoded_Bound(Input: System.Address; Len: Interfaces.Integer_64)
			return Interfaces.Integer_64;
	pragma Import(C, C_Decoded_Bound, "lz4ada_decoded_bound");

	function C_Decode_Frame_Multi(Frame: System.Address; Len: Interfaces.Integer_64;
			N_GPUs: Interfaces.Integer_32; Devices: System.Address;
			Out_Buf: System.Address; Out_Cap: Interfaces.Integer_64;
			Out_Len, Consumed: access Interfaces.Integer_64)
			return Interfaces.Integer_32;
	pragma Import(C, C_Decode_Frame_Multi, "lz4ada_decode_frame_multi");

end LZ4Ada.GPU;
