// Command gpuminer is a GPU-backed miner for the unchanged reference server:
// it speaks the same LSP protocol and bitcoin.Message contract as
// cmu440/bitcoin/miner (Join, then Request -> Result), but the scan runs in
// libhipminer.so through package hipminer.
//
// Usage: gpuminer <host:port>     (HIPMINER_DEVICES=0,1,... selects GPUs)
// Build (GOPATH mode: the reference's p1/ and this repo's go/ as GOPATH entries):
//
//	GO111MODULE=off GOPATH=<reference>/p1:<repo>/go go build gpuminer
package main

import (
	"encoding/json"
	"fmt"
	"os"
	"strconv"
	"strings"

	"github.com/cmu440/bitcoin"
	"github.com/cmu440/lsp"

	"hipminer"
)

func devicesFromEnv() []int {
	var ds []int
	for _, f := range strings.Split(os.Getenv("HIPMINER_DEVICES"), ",") {
		if n, err := strconv.Atoi(strings.TrimSpace(f)); err == nil {
			ds = append(ds, n)
		}
	}
	return ds
}

// serve answers Requests until the connection fails; a GPU failure ends the
// process (no CPU fallback): the server then reassigns the chunk.
func serve(conn lsp.Client, gpu *hipminer.Miner) error {
	for {
		payload, err := conn.Read()
		if err != nil {
			return err
		}
		var req bitcoin.Message
		_ = json.Unmarshal(payload, &req) // the reference ignores decode errors
		h, n, err := gpu.EvalRequest(req.Data, req.Lower, req.Upper)
		if err != nil {
			return err
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
	if err != nil {
		fmt.Println("GPU init failed:", err)
		return
	}
	defer gpu.Close()
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
	if err := serve(conn, gpu); err != nil {
		fmt.Fprintln(os.Stderr, "gpuminer:", err)
	}
}
