// Command gpuminer is a GPU-backed miner for the unchanged reference server:
// it speaks the same LSP protocol and bitcoin.Message contract as
// cmu440/bitcoin/miner (Join, then Request -> Result), but the scan runs in
// libhipminer.so through package hipminer.
//
// Usage: gpuminer <host:port>     (HIPMINER_DEVICES=0,1,... selects GPUs;
// HM_SCAN_DEADLINE_MS bounds each GPU scan (0 = none, default auto);
// HM_MINER_RETRY_MS is the first backoff before a failed GPU is retried;
// HM_CPU_THREADS sizes the host scan used while no GPU works)
// Build (GOPATH mode: the reference's p1/ and this repo's go/ as GOPATH entries):
//
//	GO111MODULE=off GOPATH=<reference>/p1:<repo>/go go build gpuminer
//
// The same liveness rules as the native hm_miner (csrc/miner_main.cpp), which
// the GPU tests run; this file is not compiled in the build image (no Go).
package main

import (
	"encoding/json"
	"fmt"
	"os"
	"strconv"
	"strings"
	"time"

	"github.com/cmu440/bitcoin"
	"github.com/cmu440/lsp"

	"hipminer"
)

// devicesFromEnv parses HIPMINER_DEVICES; a malformed entry is the one fatal
// configuration error.
func devicesFromEnv() ([]int, error) {
	var ds []int
	for _, f := range strings.Split(os.Getenv("HIPMINER_DEVICES"), ",") {
		f = strings.TrimSpace(f)
		if f == "" {
			continue
		}
		n, err := strconv.Atoi(f)
		if err != nil || n < 0 {
			return nil, fmt.Errorf("bad HIPMINER_DEVICES entry %q", f)
		}
		ds = append(ds, n)
	}
	return ds, nil
}

func envInt(name string, dflt int64) int64 {
	if v, err := strconv.ParseInt(os.Getenv(name), 10, 64); err == nil {
		return v
	}
	return dflt
}

// gpu is the GPU side of the miner: an open Miner, or the time the next
// Open may be tried (backoff doubling from HM_MINER_RETRY_MS up to 60 s).
type gpu struct {
	devices  []int
	deadline int64
	backoff  time.Duration
	m        *hipminer.Miner
	retryAt  time.Time
}

func (g *gpu) open() error {
	m, err := hipminer.Open(g.devices...)
	if err == nil && g.deadline != 0 {
		if err = m.SetDeadline(g.deadline); err != nil {
			m.Close()
		}
	}
	if err != nil {
		return err
	}
	g.m = m
	return nil
}

func (g *gpu) backOff() {
	g.retryAt = time.Now().Add(g.backoff)
	g.backoff *= 2
	if g.backoff < time.Second {
		g.backoff = time.Second
	}
	if g.backoff > time.Minute {
		g.backoff = time.Minute
	}
}

// serve answers Requests until the connection fails.  A Request the GPU
// cannot answer -- no context, a failed scan, a missed deadline -- is
// answered on the host, loudly, and the GPU is retried after a backoff: a
// Result is always written, as the reference miner writes one
// (miner.go:60-62; SURVEY §8(b)).
func serve(conn lsp.Client, g *gpu, cpuThreads int) error {
	for {
		payload, err := conn.Read()
		if err != nil {
			return err
		}
		var req bitcoin.Message
		_ = json.Unmarshal(payload, &req) // the reference ignores decode errors
		if g.m == nil && !time.Now().Before(g.retryAt) {
			if err := g.open(); err != nil {
				g.backOff()
			} else {
				fmt.Fprintln(os.Stderr, "gpuminer: GPU (re)opened")
			}
		}
		var h, n uint64
		err = fmt.Errorf("no GPU")
		if g.m != nil {
			if h, n, err = g.m.EvalRequest(req.Data, req.Lower, req.Upper); err != nil {
				fmt.Fprintln(os.Stderr, "gpuminer: GPU scan FAILED:", err,
					"- this Request is scanned on the host (hm_scan_cpu); GPU retried in", g.backoff)
				g.m.Close() // after ErrTimeout: host memory only, no device wait
				g.m = nil
				g.backOff()
			}
		}
		if err != nil {
			if h, n, err = hipminer.EvalRequestCPU(req.Data, req.Lower, req.Upper, cpuThreads); err != nil {
				return err
			}
		}
		out, _ := json.Marshal(bitcoin.NewResult(h, n))
		if err := conn.Write(out); err != nil {
			return err
		}
	}
}

func main() {
	if len(os.Args) != 2 {
		fmt.Printf("Usage: ./%s <hostport>", os.Args[0])
		return
	}
	devs, err := devicesFromEnv()
	if err != nil {
		fmt.Println(err)
		return
	}
	g := &gpu{devices: devs, deadline: envInt("HM_SCAN_DEADLINE_MS", hipminer.DeadlineAuto),
		backoff: time.Duration(envInt("HM_MINER_RETRY_MS", 1000)) * time.Millisecond}
	if err := g.open(); err != nil {
		fmt.Fprintln(os.Stderr, "gpuminer: NO GPU:", err,
			"- Requests are scanned on the host (hm_scan_cpu); hipminer.Open is retried with backoff")
		g.backOff()
	}
	cpuThreads, _ := strconv.Atoi(os.Getenv("HM_CPU_THREADS"))
	conn, err := lsp.NewClient(os.Args[1], lsp.NewParams())
	if err != nil {
		fmt.Println("Failed to join with server:", err)
		return
	}
	defer conn.Close()
	join, _ := json.Marshal(bitcoin.NewJoin())
	if err := conn.Write(join); err != nil {
		return
	}
	err = serve(conn, g, cpuThreads)
	if g.m != nil {
		g.m.Close()
	}
	if err != nil {
		fmt.Fprintln(os.Stderr, "gpuminer:", err)
	}
}
