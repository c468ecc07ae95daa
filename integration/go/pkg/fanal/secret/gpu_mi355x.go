//go:build mi355x

// GPU backend of the secret scanner: the MI355X engine behind the C ABI of
// include/trivy_secret_gpu.h (libtrivy_secret_gpu.so).  Compiled only with
// `go build -tags mi355x`; the pure-Go Scanner stays the default.
//
// Executable mirror: trivy_amd/secret.py (Scanner, Batch) and its tests.
package secret

/*
#cgo CFLAGS: -I${SRCDIR}/../../../third_party/trivy_amd/include
#cgo LDFLAGS: -L${SRCDIR}/../../../third_party/trivy_amd/lib -ltrivy_secret_gpu -Wl,-rpath,$ORIGIN
#include <stdlib.h>
#include "trivy_secret_gpu.h"
*/
import "C"

import (
	"runtime"
	"sync"
	"unsafe"

	"golang.org/x/xerrors"

	"github.com/aquasecurity/trivy/pkg/fanal/types"
)

// GPUBackend is one compiled ruleset (NewScanner's Global, scanner.go:315-359)
// on one engine (one GPU, one HIP stream).  Calls on it are serialised.
type GPUBackend struct {
	mu      sync.Mutex
	engine  *C.tsg_engine
	ruleset *C.tsg_ruleset
	rules   []Rule // same order as passed to tsg_ruleset_compile
}

func lastError(what string) error {
	return xerrors.Errorf("%s: %s", what, C.GoString(C.tsg_last_error()))
}

// cstrs keeps C copies alive for the duration of a call (cgo forbids
// retaining Go pointers; the library copies everything it keeps).
type cstrs []unsafe.Pointer

func (c *cstrs) str(s string) *C.char {
	p := C.CString(s)
	*c = append(*c, unsafe.Pointer(p))
	return p
}

func (c *cstrs) opt(r *Regexp) *C.char {
	if r == nil || r.Regexp == nil {
		return nil
	}
	return c.str(r.String())
}

func (c *cstrs) alloc(n int, size uintptr) unsafe.Pointer {
	p := C.calloc(C.size_t(n+1), C.size_t(size))
	*c = append(*c, p)
	return p
}

func (c *cstrs) free() {
	for _, p := range *c {
		C.free(p)
	}
}

// NewGPUBackend compiles s's rules (builtin ∪ custom, already filtered by
// NewScanner) for GPU `device` and creates the device's engine.  It fails
// with TSG_ERR_NO_DEVICE on a host without a usable GPU and with
// TSG_ERR_UNSUPPORTED for a rule outside the engine's coverage; every caller
// in the mi355x build (analyzer/secret/secret_mi355x.go, the image-config and
// layer hooks) then keeps Trivy's pure-Go Scanner.  Close frees the engine
// (a finalizer does it too, for a backend nobody closed).
func NewGPUBackend(s Scanner, device int) (*GPUBackend, error) {
	g := s.Global
	var keep cstrs
	defer keep.free()
	crules := make([]C.tsg_rule, len(g.Rules)+1)
	for i, r := range g.Rules {
		kws := unsafe.Slice((**C.char)(keep.alloc(len(r.Keywords), unsafe.Sizeof(uintptr(0)))), len(r.Keywords)+1)
		for k, kw := range r.Keywords {
			kws[k] = keep.str(kw)
		}
		ars := unsafe.Slice((*C.tsg_allow_rule)(keep.alloc(len(r.AllowRules), unsafe.Sizeof(C.tsg_allow_rule{}))),
			len(r.AllowRules)+1)
		for k, a := range r.AllowRules {
			ars[k] = C.tsg_allow_rule{id: keep.str(a.ID), regex: keep.opt(a.Regex), path: keep.opt(a.Path)}
		}
		exs := unsafe.Slice((**C.char)(keep.alloc(len(r.ExcludeBlock.Regexes), unsafe.Sizeof(uintptr(0)))),
			len(r.ExcludeBlock.Regexes)+1)
		for k, x := range r.ExcludeBlock.Regexes {
			exs[k] = keep.opt(x)
		}
		crules[i] = C.tsg_rule{
			id: keep.str(r.ID), regex: keep.opt(r.Regex),
			keywords: &kws[0], n_keywords: C.size_t(len(r.Keywords)),
			path: keep.opt(r.Path), secret_group_name: keep.str(r.SecretGroupName),
			allow_rules: &ars[0], n_allow_rules: C.size_t(len(r.AllowRules)),
			exclude_regexes: &exs[0], n_exclude_regexes: C.size_t(len(r.ExcludeBlock.Regexes)),
		}
	}
	gar := unsafe.Slice((*C.tsg_allow_rule)(keep.alloc(len(g.AllowRules), unsafe.Sizeof(C.tsg_allow_rule{}))),
		len(g.AllowRules)+1)
	for k, a := range g.AllowRules {
		gar[k] = C.tsg_allow_rule{id: keep.str(a.ID), regex: keep.opt(a.Regex), path: keep.opt(a.Path)}
	}
	gex := unsafe.Slice((**C.char)(keep.alloc(len(g.ExcludeBlock.Regexes), unsafe.Sizeof(uintptr(0)))),
		len(g.ExcludeBlock.Regexes)+1)
	for k, x := range g.ExcludeBlock.Regexes {
		gex[k] = keep.opt(x)
	}
	b := &GPUBackend{rules: g.Rules}
	if rc := C.tsg_engine_create(C.int(device), &b.engine); rc != C.TSG_OK {
		return nil, lastError("mi355x engine")
	}
	var errbuf [1024]C.char
	if rc := C.tsg_ruleset_compile(&crules[0], C.size_t(len(g.Rules)), &gar[0], C.size_t(len(g.AllowRules)),
		&gex[0], C.size_t(len(g.ExcludeBlock.Regexes)), &b.ruleset, &errbuf[0], C.size_t(len(errbuf))); rc != C.TSG_OK {
		C.tsg_engine_free(b.engine)
		return nil, xerrors.Errorf("regexp compile error: %s", C.GoString(&errbuf[0]))
	}
	runtime.SetFinalizer(b, (*GPUBackend).Close)
	return b, nil
}

// Close frees the ruleset and the engine (its device memory); safe to call
// twice.
func (b *GPUBackend) Close() {
	b.mu.Lock()
	defer b.mu.Unlock()
	if b.ruleset != nil {
		C.tsg_ruleset_free(b.ruleset)
		b.ruleset = nil
	}
	if b.engine != nil {
		C.tsg_engine_free(b.engine)
		b.engine = nil
	}
}

// Batch is a caller-filled, page-locked staging buffer (tsg_staging_*):
// files are read straight into it, so a batch costs one host write per byte
// and one host-to-device copy.
type Batch struct {
	b     *GPUBackend
	st    *C.tsg_staging
	paths []string
	slots [][]byte // each file's region of the staging buffer (C memory)
}

// NewBatch allocates a staging buffer of `capacity` bytes (contents + one
// separator byte per file).
func (b *GPUBackend) NewBatch(capacity int) (*Batch, error) {
	t := &Batch{b: b}
	if rc := C.tsg_staging_create(C.size_t(capacity), &t.st); rc != C.TSG_OK {
		return nil, lastError("mi355x staging")
	}
	return t, nil
}

// Len is the number of files added since the last run.
func (t *Batch) Len() int { return len(t.paths) }

// Reserve reserves `size` bytes for filePath and returns that region of the
// staging buffer (C memory: the caller reads the file into it, e.g.
// io.ReadFull, before the batch runs).  ok is false when the buffer has no
// room: run the batch and reserve again; a file larger than the whole buffer
// never fits (use AnalyzeBatch / ScanBatch).  A slot holds whatever an
// earlier batch left there until it is written: a caller that cannot fill it
// must clear it (NUL bytes: utils.IsBinary skips the file).
func (t *Batch) Reserve(filePath string, size int) (dst []byte, ok bool, err error) {
	cpath := C.CString(filePath)
	defer C.free(unsafe.Pointer(cpath))
	var p *C.uint8_t
	switch rc := C.tsg_staging_add(t.st, cpath, C.uint64_t(size), &p); rc {
	case C.TSG_OK:
	case C.TSG_ERR_FULL:
		return nil, false, nil
	default:
		return nil, false, lastError("mi355x staging")
	}
	if size > 0 {
		dst = unsafe.Slice((*byte)(unsafe.Pointer(p)), size)
	}
	t.paths = append(t.paths, filePath)
	t.slots = append(t.slots, dst)
	return dst, true, nil
}

// Add is Reserve followed by fill(dst); a fill error clears the slot (it
// stays in the batch and scans as binary) and is returned.
func (t *Batch) Add(filePath string, size int, fill func(dst []byte) error) (ok bool, err error) {
	dst, ok, err := t.Reserve(filePath, size)
	if err != nil || !ok {
		return ok, err
	}
	if len(dst) > 0 {
		if err := fill(dst); err != nil {
			clear(dst)
			return true, err
		}
	}
	return true, nil
}

// Content is file i's staged bytes (valid until the batch runs or resets).
func (t *Batch) Content(i int) []byte { return t.slots[i] }

// Reset empties the batch without running it.
func (t *Batch) Reset() {
	C.tsg_staging_reset(t.st)
	t.paths = t.paths[:0]
	t.slots = t.slots[:0]
}

// Analyze runs SecretAnalyzer.Analyze's per-file work (secret.go:79-113:
// IsBinary, "\r" strip, Scan) over the staged RAW files in one GPU call and
// resets the batch.  One types.Secret per added file, in order; a binary file
// or a file without findings is types.Secret{}.
func (t *Batch) Analyze() ([]types.Secret, error) { return t.run(true) }

// Scan is Scanner.Scan over the staged (already CR-stripped) contents.
func (t *Batch) Scan() ([]types.Secret, error) { return t.run(false) }

// run: one staged call.  On success the batch is reset; on an error the
// staged files stay (Content) until the caller resets it.
func (t *Batch) run(analyze bool) ([]types.Secret, error) {
	b := t.b
	b.mu.Lock()
	defer b.mu.Unlock()
	if b.engine == nil {
		return nil, xerrors.New("mi355x scan: backend closed")
	}
	var res *C.tsg_result
	var rc C.int
	if analyze { // (cgo: C functions are not Go values, so no func variable here)
		rc = C.tsg_analyze_staged(b.engine, b.ruleset, t.st, &res)
	} else {
		rc = C.tsg_scan_staged(b.engine, b.ruleset, t.st, &res)
	}
	if rc != C.TSG_OK {
		return nil, lastError("mi355x scan")
	}
	defer C.tsg_result_free(res)
	out := b.convert(res, t.paths)
	t.Reset()
	return out, nil
}

// Close frees the staging buffer.
func (t *Batch) Close() {
	if t.st != nil {
		C.tsg_staging_free(t.st)
		t.st = nil
	}
}

// ScanBatch is Scan over many in-memory files in one GPU pass (each content
// copied once, into the staging buffer).  Each result equals what
// (*Scanner).Scan returns for that file.
func (b *GPUBackend) ScanBatch(args []ScanArgs) ([]types.Secret, error) { return b.batchOf(args, false) }

// AnalyzeBatch is SecretAnalyzer.Analyze's per-file work (IsBinary, "\r"
// strip, Scan) over RAW in-memory files in one GPU pass.
func (b *GPUBackend) AnalyzeBatch(args []ScanArgs) ([]types.Secret, error) { return b.batchOf(args, true) }

func (b *GPUBackend) batchOf(args []ScanArgs, analyze bool) ([]types.Secret, error) {
	total := 1
	for _, a := range args {
		total += len(a.Content) + 1
	}
	t, err := b.NewBatch(total)
	if err != nil {
		return nil, err
	}
	defer t.Close()
	for _, a := range args {
		dst, _, err := t.Reserve(a.FilePath, len(a.Content))
		if err != nil {
			return nil, err
		}
		copy(dst, a.Content)
	}
	return t.run(analyze)
}

// convert turns a result into types.Secret values (scanner.go:436-451):
// findings in Scan order, rule metadata from the host's rules.
func (b *GPUBackend) convert(res *C.tsg_result, paths []string) []types.Secret {
	out := make([]types.Secret, len(paths))
	if len(paths) == 0 {
		return out
	}
	flags := unsafe.Slice(C.tsg_result_file_flags(res), len(paths))
	for i, p := range paths {
		if flags[i]&C.TSG_FILE_BINARY != 0 {
			continue // Analyze: utils.IsBinary -> nil (secret.go:80-84)
		}
		if flags[i]&C.TSG_FILE_PATH_ALLOWED != 0 {
			out[i] = types.Secret{FilePath: p} // scanner.go:375-379
			continue
		}
		var fp *C.tsg_finding
		n := int(C.tsg_result_findings(res, C.size_t(i), &fp))
		if n == 0 {
			continue // types.Secret{} (scanner.go:437-439)
		}
		sec := types.Secret{FilePath: p}
		for _, f := range unsafe.Slice(fp, n) {
			r := b.rules[f.rule]
			var code types.Code
			if f.n_lines > 0 {
				for _, l := range unsafe.Slice(f.lines, int(f.n_lines)) {
					s := C.GoStringN(l.content, C.int(l.content_len))
					code.Lines = append(code.Lines, types.Line{Number: int(l.number), Content: s, Highlighted: s,
						IsCause: l.is_cause != 0, FirstCause: l.first_cause != 0, LastCause: l.last_cause != 0})
				}
			}
			sev := r.Severity
			if sev == "" {
				sev = "UNKNOWN"
			}
			sec.Findings = append(sec.Findings, types.SecretFinding{RuleID: r.ID, Category: r.Category,
				Severity: sev, Title: r.Title, StartLine: int(f.start_line), EndLine: int(f.end_line),
				Code: code, Match: C.GoStringN(f.match, C.int(f.match_len))})
		}
		out[i] = sec
	}
	return out
}

// AnalyzeLayer is the secret analyzer over one decompressed image layer in
// memory (C memory, e.g. the layer read or mmap'd outside the Go heap):
// LayerTar.Walk (walker/tar.go:35-117) natively, then Required + Analyze of
// every regular file in one GPU call (tsg_analyze_layer; paths "/"-prefixed
// as Analyze does for Dir "", secret.go:95-98).  Returns the secrets with
// findings (the caller's AnalysisResult.Sort orders them, analyzer.go:218-229),
// the opaque dirs and the whiteout files.
func (b *GPUBackend) AnalyzeLayer(layer unsafe.Pointer, n int, skipFiles, skipDirs []string,
	configPath string) ([]types.Secret, []string, []string, error) {
	var keep cstrs
	defer keep.free()
	sf := unsafe.Slice((**C.char)(keep.alloc(len(skipFiles), unsafe.Sizeof(uintptr(0)))), len(skipFiles)+1)
	for i, s := range skipFiles {
		sf[i] = keep.str(s)
	}
	sd := unsafe.Slice((**C.char)(keep.alloc(len(skipDirs), unsafe.Sizeof(uintptr(0)))), len(skipDirs)+1)
	for i, s := range skipDirs {
		sd[i] = keep.str(s)
	}
	var w *C.tsg_tar_walk
	if rc := C.tsg_layer_tar_walk((*C.uint8_t)(layer), C.size_t(n), &sf[0], C.size_t(len(skipFiles)), &sd[0],
		C.size_t(len(skipDirs)), &w); rc != C.TSG_OK {
		return nil, nil, nil, xerrors.New(C.GoString(C.tsg_last_error())) // "failed to extract the archive: ..."
	}
	defer C.tsg_tar_walk_free(w)
	var opq, wh []string
	for i := 0; i < int(C.tsg_tar_walk_opq_count(w)); i++ {
		opq = append(opq, C.GoString(C.tsg_tar_walk_opq_dir(w, C.size_t(i))))
	}
	for i := 0; i < int(C.tsg_tar_walk_wh_count(w)); i++ {
		wh = append(wh, C.GoString(C.tsg_tar_walk_wh_file(w, C.size_t(i))))
	}
	ne := int(C.tsg_tar_walk_entry_count(w))
	kept := make([]C.uint32_t, ne+1)
	var nk C.size_t
	var res *C.tsg_result
	b.mu.Lock()
	if b.engine == nil {
		b.mu.Unlock()
		return nil, nil, nil, xerrors.New("secret scan error: backend closed")
	}
	rc := C.tsg_analyze_layer(b.engine, b.ruleset, (*C.uint8_t)(layer), C.size_t(n), w, keep.str(configPath),
		&kept[0], &nk, &res)
	b.mu.Unlock()
	if rc != C.TSG_OK {
		return nil, nil, nil, lastError("secret scan error")
	}
	defer C.tsg_result_free(res)
	ents := unsafe.Slice(C.tsg_tar_walk_entries(w), ne+1)
	paths := make([]string, int(nk))
	for k := range paths {
		e := ents[kept[k]]
		paths[k] = "/" + C.GoStringN(e.path, C.int(e.path_len))
	}
	var secrets []types.Secret
	for _, s := range b.convert(res, paths) {
		if len(s.Findings) > 0 {
			secrets = append(secrets, s)
		}
	}
	return secrets, opq, wh, nil
}
