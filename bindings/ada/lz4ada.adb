-- lz4ada.adb -- thin body: every subprogram forwards to liblz4ada_hip.so.
-- UNTESTED (no GNAT in this image).  Link with -llz4ada_hip.
with Interfaces.C;
with Interfaces.C.Strings;

package body LZ4Ada is

	use Interfaces;
	package C renames Interfaces.C;
	package CS renames Interfaces.C.Strings;

	------------------------------------------------------ C entry points --

	function C_Init(Res: C.int; Min_Buf: access Integer_64;
			Ctx: access System.Address) return C.int;
	pragma Import(C, C_Init, "lz4ada_init");

	function C_Init_With_Header(Input: System.Address; Len: Integer_64;
			Res: C.int; Consumed, Min_Buf: access Integer_64;
			Ctx: access System.Address) return C.int;
	pragma Import(C, C_Init_With_Header, "lz4ada_init_with_header");

	function C_Init_For_Block(Clen: Integer_64; Res: C.int;
			Min_Buf: access Integer_64;
			Ctx: access System.Address) return C.int;
	pragma Import(C, C_Init_For_Block, "lz4ada_init_for_block");

	function C_Update(Ctx: System.Address; Input: System.Address;
			Len: Integer_64; Consumed: access Integer_64;
			Buf: System.Address; Buf_Len: Integer_64;
			First, Last: access Integer_64) return C.int;
	pragma Import(C, C_Update, "lz4ada_update");

	function C_Is_End_Of_Frame(Ctx: System.Address) return C.int;
	pragma Import(C, C_Is_End_Of_Frame, "lz4ada_is_end_of_frame");

	function C_Last_Error(Ctx: System.Address) return CS.chars_ptr;
	pragma Import(C, C_Last_Error, "lz4ada_last_error");

	function C_Thread_Last_Error return CS.chars_ptr;
	pragma Import(C, C_Thread_Last_Error, "lz4ada_thread_last_error");

	procedure C_Free(Ctx: System.Address);
	pragma Import(C, C_Free, "lz4ada_free");

	-- Map a C status to the reference exception (include/lz4ada_hip.h).
	procedure Check(Status: C.int; Msg: CS.chars_ptr) is
		Text: constant String := (if Msg = CS.Null_Ptr then ""
							else CS.Value(Msg));
	begin
		case Status is
		when 0 => null;
		when 1 => raise Checksum_Error with Text;
		when 2 => raise Data_Corruption with Text;
		when 3 => raise Not_Supported with Text;
		when 4 => raise Too_Few_Header_Bytes with Text;
		when 5 => raise Too_Little_Memory with Text;
		when 6 => raise Program_Error with Text;  -- Assertion_Error
		when 7 => raise Constraint_Error with Text;
		when others => raise Device_Error with Text;
		end case;
	end Check;

	function Wrap(Handle: System.Address; Min: Integer_64)
						return Decompressor is
	begin
		return D: Decompressor(In_Last => Integer(Min)) do
			D.Handle := Handle;
		end return;
	end Wrap;

	overriding procedure Finalize(Ctx: in out Decompressor) is
	begin
		if Ctx.Handle /= System.Null_Address then
			C_Free(Ctx.Handle);
			Ctx.Handle := System.Null_Address;
		end if;
	end Finalize;

	------------------------------------------------------ Init variants --

	function Init(Min_Buffer_Size:   out    Ada.Streams.Stream_Element_Offset;
			Reservation:     in     Memory_Reservation := For_All)
			return Decompressor is
		Min: aliased Integer_64;
		H:   aliased System.Address;
	begin
		Check(C_Init(Memory_Reservation'Pos(Reservation), Min'Access,
					H'Access), C_Thread_Last_Error);
		Min_Buffer_Size := Ada.Streams.Stream_Element_Offset(Min);
		return Wrap(H, Min);
	end Init;

	function Init(Min_Buffer_Size:   out    Integer;
			Reservation:     in     Memory_Reservation := For_All)
			return Decompressor is
		Min: aliased Integer_64;
		H:   aliased System.Address;
	begin
		Check(C_Init(Memory_Reservation'Pos(Reservation), Min'Access,
					H'Access), C_Thread_Last_Error);
		Min_Buffer_Size := Integer(Min);
		return Wrap(H, Min);
	end Init;

	function Init_With_Header(Input: in     Octets;
			Num_Consumed:    out    Integer;
			Min_Buffer_Size: out    Integer;
			Reservation:     in     Flexible_Memory_Reservation
								:= Single_Frame)
			return Decompressor is
		Used, Min: aliased Integer_64;
		H:         aliased System.Address;
	begin
		Check(C_Init_With_Header(Input'Address, Input'Length,
			Flexible_Memory_Reservation'Pos(Reservation), Used'Access,
			Min'Access, H'Access), C_Thread_Last_Error);
		Num_Consumed    := Integer(Used);
		Min_Buffer_Size := Integer(Min);
		return Wrap(H, Min);
	end Init_With_Header;

	function Init_For_Block(Min_Buffer_Size:  out Integer;
				Compressed_Length: in Integer;
				Reservation:       in Memory_Reservation
						:= For_All) return Decompressor is
		Min: aliased Integer_64;
		H:   aliased System.Address;
	begin
		Check(C_Init_For_Block(Integer_64(Compressed_Length),
			Memory_Reservation'Pos(Reservation), Min'Access,
			H'Access), C_Thread_Last_Error);
		Min_Buffer_Size := Integer(Min);
		return Wrap(H, Min);
	end Init_For_Block;

	------------------------------------------------------------ Update --

	procedure Update(Ctx:            in out Decompressor;
			Input:           in     Ada.Streams.Stream_Element_Array;
			Num_Consumed:    out    Ada.Streams.Stream_Element_Offset;
			Buffer:          in out Ada.Streams.Stream_Element_Array;
			Output_First:    out    Ada.Streams.Stream_Element_Offset;
			Output_Last:     out    Ada.Streams.Stream_Element_Offset) is
		use type Ada.Streams.Stream_Element_Offset;
		Used, First, Last: aliased Integer_64;
	begin
		Check(C_Update(Ctx.Handle, Input'Address, Input'Length,
			Used'Access, Buffer'Address, Buffer'Length,
			First'Access, Last'Access), C_Last_Error(Ctx.Handle));
		-- C indices are 0-based into Buffer.
		Num_Consumed := Ada.Streams.Stream_Element_Offset(Used);
		if Last < First then
			Output_First := Buffer'First + 1;
			Output_Last  := Buffer'First;
		else
			Output_First := Buffer'First +
					Ada.Streams.Stream_Element_Offset(First);
			Output_Last  := Buffer'First +
					Ada.Streams.Stream_Element_Offset(Last);
		end if;
	end Update;

	procedure Update(Ctx:            in out Decompressor;
			Input:           in     Octets;
			Num_Consumed:    out    Integer;
			Buffer:          in out Octets;
			Output_First:    out    Integer;
			Output_Last:     out    Integer) is
		Used, First, Last: aliased Integer_64;
	begin
		Check(C_Update(Ctx.Handle, Input'Address, Input'Length,
			Used'Access, Buffer'Address, Buffer'Length,
			First'Access, Last'Access), C_Last_Error(Ctx.Handle));
		Num_Consumed := Integer(Used);
		Output_First := Integer(First);
		Output_Last  := Integer(Last);
	end Update;

	function Is_End_Of_Frame(Ctx: in Decompressor) return End_Of_Frame is
	begin
		return End_Of_Frame'Val(C_Is_End_Of_Frame(Ctx.Handle));
	end Is_End_Of_Frame;

	------------------------------------------------------------ To_Hex --

	procedure C_Hex8(V: U8; Out_Buf: out C.char_array);
	pragma Import(C, C_Hex8, "lz4ada_to_hex8");
	procedure C_Hex32(V: U32; Out_Buf: out C.char_array);
	pragma Import(C, C_Hex32, "lz4ada_to_hex32");

	function To_Hex(Num: in U8) return String is
		B: C.char_array(0 .. 2);
	begin
		C_Hex8(Num, B);
		return C.To_Ada(B);
	end To_Hex;

	function To_Hex(Num: in U32) return String is
		B: C.char_array(0 .. 8);
	begin
		C_Hex32(Num, B);
		return C.To_Ada(B);
	end To_Hex;

	---------------------------------------------------------- XXHash32 --

	package body XXHash32 is

		procedure C_X_Init(H: in out Hasher; Seed: U32);
		pragma Import(C, C_X_Init, "lz4ada_xxh32_init");
		procedure C_X_Reset(H: in out Hasher; Seed: U32);
		pragma Import(C, C_X_Reset, "lz4ada_xxh32_reset");
		function C_X_Update(H: access Hasher; Data: System.Address;
					Len: Integer_64) return C.int;
		pragma Import(C, C_X_Update, "lz4ada_xxh32_update");
		function C_X_Final(H: access constant Hasher) return U32;
		pragma Import(C, C_X_Final, "lz4ada_xxh32_final");

		function Init(Seed: in U32 := 0) return Hasher is
		begin
			return H: Hasher do
				C_X_Init(H, Seed);  -- Seed ignored (quirk Q1)
			end return;
		end Init;

		procedure Reset(Ctx: in out Hasher; Seed: in U32 := 0) is
		begin
			C_X_Reset(Ctx, Seed);
		end Reset;

		procedure Update(Ctx: in out Hasher; Input: in Octets) is
			H: aliased Hasher with Import, Address => Ctx'Address;
		begin
			Check(C_X_Update(H'Access, Input'Address, Input'Length),
							C_Thread_Last_Error);
		end Update;

		function Final(Ctx: in Hasher) return U32 is
			H: aliased constant Hasher
					with Import, Address => Ctx'Address;
		begin
			return C_X_Final(H'Access);
		end Final;

		function Hash(Input: in Octets) return U32 is
			H: Hasher := Init;
		begin
			Update(H, Input);
			return Final(H);
		end Hash;

	end XXHash32;

end LZ4Ada;
