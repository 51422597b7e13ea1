//go:build kungfu_amd

// Known answers of the reference's own tests, through the HIP drop-in:
// test_kungfu.cpp:11-20 (1 + 2 = 3), test_operations.cpp:3-26 (the four ops),
// plus integer wrap and fp16 rounding as the reference computes them
// (op.cpp:22-54, f16.c:16-50). Needs a gfx950 device.
package base

import (
	"encoding/binary"
	"math"
	"testing"
)

func f32Vector(xs ...float32) *Vector {
	v := NewVector(len(xs), F32)
	for i, x := range xs {
		binary.LittleEndian.PutUint32(v.Data[4*i:], math.Float32bits(x))
	}
	return v
}

func f32At(v *Vector, i int) float32 {
	return math.Float32frombits(binary.LittleEndian.Uint32(v.Data[4*i:]))
}

func TestTransform2OnePlusTwo(t *testing.T) {
	x, y := f32Vector(1), f32Vector(2)
	Transform2(x, x, y, SUM) // out aliases input 1, as test_kungfu.cpp does
	if got := f32At(x, 0); got != 3 {
		t.Fatalf("1 + 2 = %v", got)
	}
}

func TestTransformOps(t *testing.T) {
	want := map[OP][]float32{
		SUM:  {5, 7, 9},
		MIN:  {1, 2, 3},
		MAX:  {4, 5, 6},
		PROD: {4, 10, 18},
	}
	for op, w := range want {
		x, y := f32Vector(1, 2, 3), f32Vector(4, 5, 6)
		z := NewVector(3, F32)
		Transform2(z, x, y, op)
		for i := range w {
			if got := f32At(z, i); got != w[i] {
				t.Fatalf("op %d [%d]: %v != %v", op, i, got, w[i])
			}
		}
	}
}

func TestInt32Wraps(t *testing.T) {
	x, y := NewVector(1, I32), NewVector(1, I32)
	binary.LittleEndian.PutUint32(x.Data, math.MaxInt32)
	binary.LittleEndian.PutUint32(y.Data, 1)
	Transform(x, y, SUM)
	if got := int32(binary.LittleEndian.Uint32(x.Data)); got != math.MinInt32 {
		t.Fatalf("MaxInt32 + 1 = %d", got)
	}
}

func TestFloat16RoundsToNearestEven(t *testing.T) {
	// 2048 + 1 is a tie in binary16 (spacing 2 above 2048): RNE keeps 2048
	x, y, z := NewVector(9, F16), NewVector(9, F16), NewVector(9, F16)
	for i := 0; i < 9; i++ { // 9 elements: one 8-wide batch + a tail of 1
		binary.LittleEndian.PutUint16(x.Data[2*i:], 0x6800) // 2048
		binary.LittleEndian.PutUint16(y.Data[2*i:], 0x3c00) // 1
	}
	Transform2(z, x, y, SUM)
	for i := 0; i < 9; i++ {
		if got := binary.LittleEndian.Uint16(z.Data[2*i:]); got != 0x6800 {
			t.Fatalf("[%d] 2048 + 1 = %#04x", i, got)
		}
	}
}

func TestTypeSizes(t *testing.T) {
	for dt, sz := range map[DataType]int{U8: 1, I16: 2, F16: 2, BF16: 2, F32: 4, I64: 8, F64: 8} {
		if dt.Size() != sz {
			t.Fatalf("%s: size %d", dt, dt.Size())
		}
	}
}
