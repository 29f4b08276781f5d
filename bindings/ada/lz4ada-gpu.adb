-- lz4ada-gpu.adb -- UNTESTED (no GNAT in this image).
with Interfaces.C.Strings;

package body LZ4Ada.GPU is

	use type Interfaces.Integer_32;

	function C_Thread_Last_Error return Interfaces.C.Strings.chars_ptr;
	pragma Import(C, C_Thread_Last_Error, "lz4ada_thread_last_error");

	procedure Check(Status: Interfaces.Integer_32) is
		Text: constant String :=
			Interfaces.C.Strings.Value(C_Thread_Last_Error);
	begin
		case Status is
		when 0 => null;
		when 1 => raise Checksum_Error with Text;
		when 2 => raise Data_Corruption with Text;
		when 3 => raise Not_Supported with Text;
		when 4 => raise Too_Few_Header_Bytes with Text;
		when 5 => raise Too_Little_Memory with Text;
		when 6 => raise Program_Error with Text;
		when 7 => raise Constraint_Error with Text;
		when others => raise Device_Error with Text;
		end case;
	end Check;

	procedure Decode_Frame(Frame:          in     Octets;
				Output:         in out Octets;
				Output_Length:  out    Interfaces.Integer_64;
				Frame_Consumed: out    Interfaces.Integer_64) is
		L, C: aliased Interfaces.Integer_64;
	begin
		Check(C_Decode_Frame(Frame'Address, Frame'Length,
			Output'Address, Output'Length, L'Access, C'Access));
		Output_Length  := L;
		Frame_Consumed := C;
	end Decode_Frame;

	procedure Decode_Stream(Input:         in     Octets;
				Output:        in out Octets;
				Output_Length: out    Interfaces.Integer_64) is
		L: aliased Interfaces.Integer_64;
	begin
		Check(C_Decode_Stream(Input'Address, Input'Length,
			Output'Address, Output'Length, L'Access));
		Output_Length := L;
	end Decode_Stream;

	function Decoded_Bound(Input: in Octets) return Interfaces.Integer_64 is
	begin
		return C_Decoded_Bound(Input'Address, Input'Length);
	end Decoded_Bound;

	procedure Decode_Frame_Multi(Frame:          in     Octets;
				N_GPUs:         in     Positive;
				Output:         in out Octets;
				Output_Length:  out    Interfaces.Integer_64;
				Frame_Consumed: out    Interfaces.Integer_64) is
		L, C: aliased Interfaces.Integer_64;
	begin
		Check(C_Decode_Frame_Multi(Frame'Address, Frame'Length,
			Interfaces.Integer_32(N_GPUs), System.Null_Address,
			Output'Address, Output'Length, L'Access, C'Access));
		Output_Length  := L;
		Frame_Consumed := C;
	end Decode_Frame_Multi;

end LZ4Ada.GPU;
