// Command gpuminer is a GPU-backed miner for the unchanged reference server:
// it speaks the same LSP protocol and bitcoin.Message contract as
// cmu440/bitcoin/miner (Join, then Request -> Result), but the scan runs in
// libhipminer.so through package hipminer.
//
// Usage: gpuminer <host:port>     (HIPMINER_DEVICES=0,1,... selects GPUs;
// HM_CPU_THREADS sizes the host scan used when no GPU works)
// Build (GOPATH mode: the reference's p1/ and this repo's go/ as GOPATH entries):
//
//	GO111MODULE=off GOPATH=<reference>/p1:<repo>/go go build gpuminer
package main

import (
	"encoding/json"
	"errors"
	"fmt"
	"os"
	"strconv"
	"strings"

	"github.com/cmu440/bitcoin"
	"github.com/cmu440/lsp"

	"hipminer"
)

var errNoGPU = errors.New("no GPU")

func devicesFromEnv() []int {
	var ds []int
	for _, f := range strings.Split(os.Getenv("HIPMINER_DEVICES"), ",") {
		if n, err := strconv.Atoi(strings.TrimSpace(f)); err == nil {
			ds = append(ds, n)
		}
	}
	return ds
}

// serve answers Requests until the connection fails.  gpu == nil, or a
// failed GPU scan, sends every (later) Request to the host scan, loudly: a
// Result is always written, as the reference miner writes one
// (miner.go:60-62; SURVEY §8(b)).
func serve(conn lsp.Client, gpu *hipminer.Miner, cpuThreads int) error {
	for {
		payload, err := conn.Read()
		if err != nil {
			return err
		}
		var req bitcoin.Message
		_ = json.Unmarshal(payload, &req) // the reference ignores decode errors
		var h, n uint64
		err = errNoGPU
		if gpu != nil {
			if h, n, err = gpu.EvalRequest(req.Data, req.Lower, req.Upper); err != nil {
				fmt.Fprintln(os.Stderr, "gpuminer: GPU scan FAILED:", err,
					"- this and every later Request are scanned on the host (hm_scan_cpu)")
				gpu.Close()
				gpu = nil
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
	gpu, err := hipminer.Open(devicesFromEnv()...)
	if e, ok := err.(hipminer.Error); ok && e.Code == hipminer.ErrInvalid {
		fmt.Println("bad HIPMINER_DEVICES:", err)
		return
	}
	if err != nil {
		gpu = nil
		fmt.Fprintln(os.Stderr, "gpuminer: NO GPU:", err,
			"- every Request is scanned on the host (hm_scan_cpu), orders of magnitude slower")
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
	err = serve(conn, gpu, cpuThreads)
	if gpu != nil {
		gpu.Close()
	}
	if err != nil {
		fmt.Fprintln(os.Stderr, "gpuminer:", err)
	}
}
