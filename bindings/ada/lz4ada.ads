-- lz4ada.ads -- drop-in spec of package LZ4Ada (reference lib/lz4ada.ads)
-- over the C-ABI of liblz4ada_hip.so (include/lz4ada_hip.h).
--
-- Same package name, types, subprogram profiles and exceptions as the
-- reference spec, so callers (tool_unlz4ada, lz4test, ...) recompile
-- unchanged; the body (lz4ada.adb in this directory) forwards every call
-- through pragma Import and re-raises the C status as the matching
-- exception with the library's message text.
--
-- UNTESTED: this image has no GNAT (see DESIGN.md section 5); the binding
-- is written against the Ada 2012 RM and the C header only.
with Ada.Streams;
with Ada.Finalization;
with Interfaces;
with System;

package LZ4Ada is

	subtype U8  is Interfaces.Unsigned_8;
	subtype U32 is Interfaces.Unsigned_32;
	subtype U64 is Interfaces.Unsigned_64;
	type Octets is array (Integer range <>) of U8;

	-- lz4ada.ads:79-106; positions equal the C enum lz4ada_reservation.
	type Flexible_Memory_Reservation is (SZ_64_KiB, SZ_256_KiB, SZ_1_MiB,
				SZ_4_MiB, SZ_8_MiB, Use_First, Single_Frame);
	subtype Memory_Reservation is Flexible_Memory_Reservation range
							SZ_64_KiB .. SZ_8_MiB;
	For_Modern: constant Memory_Reservation := SZ_4_MiB;
	For_Legacy: constant Memory_Reservation := SZ_8_MiB;
	For_All:    constant Memory_Reservation := SZ_8_MiB;

	-- lz4ada.ads:124; positions equal lz4ada_end_of_frame.
	type End_Of_Frame is (Yes, No, Maybe);

	type Decompressor(In_Last: Integer) is tagged limited private;

	-- lz4ada.ads:133-162
	Checksum_Error:       exception;
	Data_Corruption:      exception;
	Not_Supported:        exception;
	Too_Few_Header_Bytes: exception;
	Too_Little_Memory:    exception;
	-- No reference twin: HIP runtime error / no usable GPU.
	Device_Error:         exception;

	function Init(Min_Buffer_Size:   out    Ada.Streams.Stream_Element_Offset;
			Reservation:     in     Memory_Reservation := For_All)
			return Decompressor;

	procedure Update(Ctx:            in out Decompressor;
			Input:           in     Ada.Streams.Stream_Element_Array;
			Num_Consumed:    out    Ada.Streams.Stream_Element_Offset;
			Buffer:          in out Ada.Streams.Stream_Element_Array;
			Output_First:    out    Ada.Streams.Stream_Element_Offset;
			Output_Last:     out    Ada.Streams.Stream_Element_Offset);

	function Init(Min_Buffer_Size:   out    Integer;
			Reservation:     in     Memory_Reservation := For_All)
			return Decompressor;

	function Init_With_Header(Input: in     Octets;
			Num_Consumed:    out    Integer;
			Min_Buffer_Size: out    Integer;
			Reservation:     in     Flexible_Memory_Reservation
								:= Single_Frame)
			return Decompressor with Pre => Input'Length >= 7;

	function Init_For_Block(Min_Buffer_Size:  out Integer;
				Compressed_Length: in Integer;
				Reservation:       in Memory_Reservation
						:= For_All) return Decompressor;

	procedure Update(Ctx:            in out Decompressor;
			Input:           in     Octets;
			Num_Consumed:    out    Integer;
			Buffer:          in out Octets;
			Output_First:    out    Integer;
			Output_Last:     out    Integer)
			with Pre => (Buffer'First = 0);

	function Is_End_Of_Frame(Ctx: in Decompressor) return End_Of_Frame;

	function To_Hex(Num: in U8)  return String;
	function To_Hex(Num: in U32) return String;

	package XXHash32 is
		type Hasher is tagged limited private;
		function  Init(Seed: in U32 := 0) return Hasher;
		procedure Reset(Ctx: in out Hasher; Seed: in U32 := 0);
		procedure Update(Ctx: in out Hasher; Input: in Octets);
		function  Final(Ctx: in Hasher) return U32;
		function  Hash(Input: in Octets) return U32;
	private
		-- Layout of lz4ada_xxh32_state (include/lz4ada_hip.h).
		type Lanes is array (0 .. 3) of U32;
		type Hasher is tagged limited record
			State:        Lanes;
			Buffer:       Octets(0 .. 15);
			Buffer_Size:  Interfaces.Integer_32;
			Hash:         U32;
			Total_Length: U64;
		end record;
		pragma Convention(C, Hasher);
	end XXHash32;

private

	type Decompressor(In_Last: Integer) is new
			Ada.Finalization.Limited_Controlled with record
		Handle: System.Address := System.Null_Address;
	end record;
	overriding procedure Finalize(Ctx: in out Decompressor);

end LZ4Ada;
