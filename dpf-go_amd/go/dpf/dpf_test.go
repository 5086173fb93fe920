package dpf

import "testing"

// Property tests in the spirit of the reference's dpf/dpf_test.go:32-73:
// the XOR of the two shares is the point function at alpha.

func TestEvalShares(t *testing.T) {
	const logN, alpha = uint64(8), uint64(123)
	a, b := Gen(alpha, logN)
	for x := uint64(0); x < 1<<logN; x++ {
		want := byte(0)
		if x == alpha {
			want = 1
		}
		if Eval(a, x, logN)^Eval(b, x, logN) != want {
			t.Fatalf("x=%d", x)
		}
	}
}

func checkFull(t *testing.T, logN, alpha uint64) {
	a, b := Gen(alpha, logN)
	fa, fb := EvalFull(a, logN), EvalFull(b, logN)
	for x := uint64(0); x < 1<<logN; x++ {
		bit := ((fa[x/8] ^ fb[x/8]) >> (x % 8)) & 1
		if (bit == 1) != (x == alpha) {
			t.Fatalf("logN=%d alpha=%d x=%d", logN, alpha, x)
		}
		if Eval(a, x, logN) != (fa[x/8]>>(x%8))&1 {
			t.Fatalf("Eval/EvalFull disagree at x=%d", x)
		}
	}
}

func TestEvalFullShares(t *testing.T)      { checkFull(t, 9, 128) }
func TestEvalFullShortShares(t *testing.T) { checkFull(t, 3, 1) }

func TestGenPanics(t *testing.T) {
	defer func() {
		if recover() == nil {
			t.Fatal("expected panic")
		}
	}()
	Gen(8, 3)
}

// Two servers' PIR answers XOR to the queried record.
func TestPirTwoServer(t *testing.T) {
	const logN = uint64(12)
	db := make([]byte, 32<<logN)
	for i := range db {
		db[i] = byte(i*131 + i>>8)
	}
	p := NewPirDB(db, logN, 1)
	defer p.Close()
	for _, alpha := range []uint64{0, 1, 777, 1<<logN - 1} {
		a, b := Gen(alpha, logN)
		ra, rb := p.Answer([]DPFkey{a}), p.Answer([]DPFkey{b})
		for j := 0; j < 32; j++ {
			if ra[0][j]^rb[0][j] != db[32*alpha+uint64(j)] {
				t.Fatalf("alpha=%d byte %d", alpha, j)
			}
		}
	}
}

func BenchmarkEvalFull20(b *testing.B) {
	k, _ := Gen(0, 20)
	b.ResetTimer()
	for i := 0; i < b.N; i++ {
		EvalFull(k, 20)
	}
}

func BenchmarkEvalFullBatch4096x20(b *testing.B) {
	keys := make([]DPFkey, 4096)
	for i := range keys {
		keys[i], _ = Gen(uint64(i), 20)
	}
	b.ResetTimer()
	for i := 0; i < b.N; i++ {
		EvalFullBatch(keys, 20, 0)
	}
}
