//go:build mi355x

// The secret analyzer of the `mi355x` build: SecretAnalyzer (secret.go) whose
// per-file Analyze stages the file for a batched GPU call instead of scanning
// it.  Executable mirror, line for line: trivy_amd/analyzer.py
// GPUSecretAnalyzer (tests/test_analyzer_group.py, tests/test_gpu_analyzer_group.py).
//
// Trivy's contract (pkg/fanal/analyzer/analyzer.go) is kept as it is:
//
//   - secrets stay a per-file analyzer.  AnalyzeFile (analyzer.go:396-448)
//     calls Required and Analyze for every file -- also the files another
//     analyzer claims (requirements.txt, pom.xml, Cargo.lock, ...), which
//     AnalyzerGroup.PostAnalyze filters out of every post-analyzer's FS
//     (analyzer.go:475-488) -- and honours the per-call disabled list (the
//     base layers of an image, image.go:209-213).
//   - Analyze reads the file straight into the process's page-locked staging
//     buffer (tsg_staging_add, no Go-heap copy) and returns.  The Analyze call
//     that finds the buffer full runs it (tsg_analyze_staged: IsBinary, the
//     "\r" strip and Scan on the GPU); each file's result is kept under its
//     os.FileInfo, the walker's value that AnalyzeFile hands to Analyze and
//     RequiredPostAnalyzers alike.
//   - A post-analyzer of the same type marks the end of each walk: its
//     Required records the walk's FileInfos (the analyzer's own predicate),
//     and PostAnalyze -- called after wg.Wait() (artifact/local/fs.go:112-118)
//     -- runs what is still staged and returns the results of exactly ITS
//     files, so artifacts analyzed at the same time never get each other's
//     secrets.  The filtered FS it receives only serves files linked through
//     --file-patterns (RequiredPostAnalyzers skips Required for those,
//     analyzer.go:457), matched with os.SameFile.
//   - Post-analyzer constructors run before the disabled check
//     (analyzer.go:358-365), so newWalkCloser creates nothing.  The GPU engine
//     is created by the first Analyze -- never for `--scanners vuln` -- and a
//     host without a usable GPU (TSG_ERR_NO_DEVICE, or a ruleset the engine
//     does not cover, TSG_ERR_UNSUPPORTED) keeps Trivy's per-file Analyze.
//   - A GPU batch that fails is re-scanned file by file from the staged bytes
//     with Trivy's Scanner: one bad batch never aborts the artifact, as
//     AnalyzeFile drops one file's error (analyzer.go:439-442).
//   - A slot the file could not be read into is cleared: NUL bytes make
//     IsBinary skip it, as the reference skips a file it cannot read, and no
//     byte of an earlier batch is ever scanned under this file's path.
//
// Image layers take artifact/image/layer_mi355x.go (one GPU call per layer).
// A layer file that reaches this analyzer anyway (its FileInfo is a tar
// header) is analyzed per file by Trivy's Analyze.
//
// Results of a walk that never reaches PostAnalyze (an artifact that failed
// half way) stay in the map until the process ends.
package secret

import (
	"archive/tar"
	"bytes"
	"context"
	"io"
	"io/fs"
	"os"
	"reflect"
	"strconv"
	"sync"

	"github.com/samber/lo"
	"golang.org/x/xerrors"

	"github.com/aquasecurity/trivy/pkg/fanal/analyzer"
	"github.com/aquasecurity/trivy/pkg/fanal/secret"
	"github.com/aquasecurity/trivy/pkg/fanal/types"
	"github.com/aquasecurity/trivy/pkg/fanal/utils"
	"github.com/aquasecurity/trivy/pkg/log"
)

const defaultGPUBatchBytes = 512 << 20 // --secret-gpu-batch-bytes

func init() {
	a := &gpuSecrets{
		SecretAnalyzer: NewSecretAnalyzer(secret.Scanner{}, ""),
		batchBytes:     defaultGPUBatchBytes,
		results:        make(map[os.FileInfo]types.Secret),
	}
	analyzer.RegisterAnalyzer(a)                                     // Required + Analyze per file
	analyzer.RegisterPostAnalyzer(analyzer.TypeSecret, a.newWalkCloser) // the end of each walk
}

// gpuDevice: the HIP ordinal of this process's GPU (one process per GPU).
func gpuDevice() int {
	if v, err := strconv.Atoi(os.Getenv("TRIVY_SECRET_GPU_DEVICE")); err == nil {
		return v
	}
	return 0
}

// stagedFile: one reserved slot of the staging buffer.
type stagedFile struct {
	info     os.FileInfo
	scanPath string // FilePath as Scan sees it ("/"-prefixed for Dir == "", secret.go:95-98)
}

// gpuSecrets is the process-wide secret analyzer of the mi355x build.
type gpuSecrets struct {
	*SecretAnalyzer
	batchBytes int

	mu      sync.Mutex // the backend, the staging buffer, batch runs
	probed  bool       // the backend was tried (first Analyze)
	gpuErr  error      // no usable GPU: Trivy's Analyze per file
	backend *secret.GPUBackend
	batch   *secret.Batch
	files   []stagedFile
	filling sync.WaitGroup // slots reserved and not yet filled (Add under mu, Wait under mu)

	rmu     sync.Mutex
	results map[os.FileInfo]types.Secret // files with findings, until their walk's PostAnalyze
}

// Init is SecretAnalyzer.Init (ParseConfig + NewScanner, secret.go:63-77).
// A new config runs what is staged with the old ruleset, then drops the
// backend; the next Analyze builds one for the new ruleset.
func (a *gpuSecrets) Init(opt analyzer.AnalyzerOptions) error {
	a.mu.Lock()
	defer a.mu.Unlock()
	oldPath, had := a.configPath, !lo.IsEmpty(a.scanner)
	if err := a.SecretAnalyzer.Init(opt); err != nil {
		return err
	}
	if had && oldPath == a.configPath {
		return nil
	}
	if a.batch != nil {
		a.runLocked()
		a.batch.Close()
		a.backend.Close()
	}
	a.probed, a.gpuErr, a.backend, a.batch = false, nil, nil, nil
	return nil
}

// backendLocked creates the engine and the staging buffer once.
func (a *gpuSecrets) backendLocked() bool {
	if !a.probed {
		a.probed = true
		be, err := secret.NewGPUBackend(a.scanner, gpuDevice())
		if err == nil {
			var b *secret.Batch
			if b, err = be.NewBatch(a.batchBytes); err == nil {
				a.backend, a.batch = be, b
			} else {
				be.Close()
			}
		}
		if err != nil {
			a.gpuErr = err
			log.Info("MI355X secret backend unavailable: Trivy's scanner analyzes each file", log.Err(err))
		}
	}
	return a.gpuErr == nil
}

// stageable: a local file whose FileInfo can key the results map (a tar
// header's goes to the per-file path).
func stageable(info os.FileInfo) bool {
	if info == nil || !reflect.TypeOf(info).Comparable() {
		return false
	}
	_, fromTar := info.Sys().(*tar.Header)
	return !fromTar
}

func (a *gpuSecrets) Analyze(ctx context.Context, input analyzer.AnalysisInput) (*analyzer.AnalysisResult, error) {
	a.mu.Lock()
	gpu := a.backendLocked()
	a.mu.Unlock()
	if !gpu || !stageable(input.Info) {
		return a.SecretAnalyzer.Analyze(ctx, input) // secret.go:79-113
	}
	// Do not scan binaries (secret.go:80-84)
	binary, err := utils.IsBinary(input.Content, input.Info.Size())
	if binary || err != nil {
		return nil, nil
	}
	f := stagedFile{info: input.Info, scanPath: input.FilePath}
	if input.Dir == "" {
		f.scanPath = "/" + input.FilePath
	}
	size := int(input.Info.Size())

	a.mu.Lock()
	dst, ok, err := a.batch.Reserve(f.scanPath, size)
	if err == nil && !ok && a.batch.Len() > 0 {
		a.runLocked() // full: this Analyze runs the batch
		dst, ok, err = a.batch.Reserve(f.scanPath, size)
	}
	if err == nil && ok {
		a.files = append(a.files, f)
		a.filling.Add(1)
	}
	a.mu.Unlock()
	if err != nil {
		return nil, err
	}
	if !ok { // larger than the whole staging buffer: this file alone
		content, err := io.ReadAll(input.Content)
		if err != nil {
			return nil, xerrors.Errorf("read error %s: %w", input.FilePath, err)
		}
		a.mu.Lock()
		out, err := a.backend.AnalyzeBatch([]secret.ScanArgs{{FilePath: f.scanPath, Content: content}})
		a.mu.Unlock()
		if err != nil {
			a.store(f.info, a.goAnalyze(f, content))
		} else {
			a.store(f.info, out[0])
		}
		return nil, nil
	}
	defer a.filling.Done()
	if _, err := io.ReadFull(input.Content, dst); err != nil {
		clear(dst)
		return nil, xerrors.Errorf("read error %s: %w", input.FilePath, err)
	}
	return nil, nil
}

// runLocked runs the staged files (caller holds mu): waits for the slots
// still being filled, one tsg_analyze_staged, results per file.  A failed
// batch is re-scanned file by file with Trivy's Scanner.
func (a *gpuSecrets) runLocked() {
	a.filling.Wait()
	files := a.files
	a.files = nil
	if len(files) == 0 {
		return
	}
	out, err := a.batch.Analyze()
	if err != nil {
		log.Debug("GPU secret batch failed: Trivy's scanner takes its files", log.Err(err))
		for i, f := range files {
			a.store(f.info, a.goAnalyze(f, a.batch.Content(i)))
		}
		a.batch.Reset()
		return
	}
	for i, f := range files {
		a.store(f.info, out[i])
	}
}

// goAnalyze is secret.go:79-113 over raw staged bytes.
func (a *gpuSecrets) goAnalyze(f stagedFile, raw []byte) types.Secret {
	if binary, err := utils.IsBinary(bytes.NewReader(raw), int64(len(raw))); binary || err != nil {
		return types.Secret{}
	}
	content := bytes.ReplaceAll(raw, []byte("\r"), []byte(""))
	return a.scanner.Scan(secret.ScanArgs{FilePath: f.scanPath, Content: content})
}

func (a *gpuSecrets) store(info os.FileInfo, s types.Secret) {
	if len(s.Findings) == 0 {
		return
	}
	a.rmu.Lock()
	a.results[info] = s
	a.rmu.Unlock()
}

// walkCloser is the post-analyzer side: one per AnalyzerGroup.
type walkCloser struct {
	owner *gpuSecrets
	mu    sync.Mutex
	infos []os.FileInfo
}

func (a *gpuSecrets) newWalkCloser(_ analyzer.AnalyzerOptions) (analyzer.PostAnalyzer, error) {
	return &walkCloser{owner: a}, nil
}

func (w *walkCloser) Type() analyzer.Type { return analyzer.TypeSecret }

func (w *walkCloser) Version() int { return version }

// Required: the analyzer's Required, recording the file.
func (w *walkCloser) Required(filePath string, info os.FileInfo) bool {
	if !stageable(info) || !w.owner.Required(filePath, info) {
		return false
	}
	w.mu.Lock()
	w.infos = append(w.infos, info)
	w.mu.Unlock()
	return true
}

func (w *walkCloser) PostAnalyze(_ context.Context, input analyzer.PostAnalysisInput) (*analyzer.AnalysisResult, error) {
	a := w.owner
	a.mu.Lock()
	if a.batch != nil {
		a.runLocked()
	}
	a.mu.Unlock()

	w.mu.Lock()
	infos := w.infos
	w.infos = nil
	w.mu.Unlock()

	var secrets []types.Secret
	a.rmu.Lock()
	for _, info := range infos {
		if s, ok := a.results[info]; ok {
			secrets = append(secrets, s)
			delete(a.results, info)
		}
	}
	more := len(a.results) > 0
	a.rmu.Unlock()

	if more { // files linked through --file-patterns
		_ = fs.WalkDir(input.FS, ".", func(p string, d fs.DirEntry, err error) error {
			if err != nil || d.IsDir() {
				return nil
			}
			fi, err := fs.Stat(input.FS, p)
			if err != nil {
				return nil
			}
			a.rmu.Lock()
			defer a.rmu.Unlock()
			for info, s := range a.results {
				if os.SameFile(info, fi) {
					secrets = append(secrets, s)
					delete(a.results, info)
					break
				}
			}
			return nil
		})
	}
	if len(secrets) == 0 {
		return nil, nil
	}
	return &analyzer.AnalysisResult{Secrets: secrets}, nil
}
