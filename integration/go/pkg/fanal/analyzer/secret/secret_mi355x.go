//go:build mi355x

// The secret analyzer of the `mi355x` build: SecretAnalyzer (secret.go) with
// its per-file Analyze replaced by a batched PostAnalyze on the GPU.
//
// Trivy calls an analyzer's Analyze once per file from the walker's goroutine
// fan-out (analyzer.go:422-444, at most --parallel files in flight), which
// cannot feed a GPU.  Registered as a PostAnalyzer instead (analyzer.go:78-82,
// RegisterPostAnalyzer :102-107), the analyzer sees each file once during the
// walk through Required -- unchanged, secret.go:115-153 -- and the artifact
// links every required file into the post-analyzer FS
// (artifact/local/fs.go:100-106).  After the walk PostAnalyze reads those
// files straight into a page-locked GPU staging buffer and runs Analyze's
// per-file work (utils.IsBinary, the "\r" strip, Scan) batch by batch, one
// tsg_analyze_staged call per --secret-gpu-batch-bytes; the secrets come back
// in one AnalysisResult that AnalyzerGroup.PostAnalyze merges (analyzer.go:468-503).
//
// Paths are the FS's relative paths, exactly what Analyze receives for a
// filesystem or repository artifact (input.Dir = the scan root, so no "/"
// prefix, secret.go:95-98).  Image layers do not reach this analyzer in the
// mi355x build: artifact/image/layer_mi355x.go analyzes each layer whole.
//
// Executable mirror, line for line: trivy_amd/analyzer.py SecretPostAnalyzer
// (tests/test_gpu_staging.py runs it against per-file Analyze and the oracle).
package secret

import (
	"context"
	"io"
	"io/fs"
	"os"
	"strconv"

	"golang.org/x/xerrors"

	"github.com/aquasecurity/trivy/pkg/fanal/analyzer"
	"github.com/aquasecurity/trivy/pkg/fanal/secret"
	"github.com/aquasecurity/trivy/pkg/fanal/types"
	"github.com/aquasecurity/trivy/pkg/log"
)

const defaultGPUBatchBytes = 512 << 20 // --secret-gpu-batch-bytes

func init() {
	analyzer.RegisterPostAnalyzer(analyzer.TypeSecret, newGPUPostAnalyzer)
}

type gpuPostAnalyzer struct {
	*SecretAnalyzer
	backend    *secret.GPUBackend
	batchBytes int
}

// gpuDevice: the HIP ordinal of this process's GPU (one process per GPU).
func gpuDevice() int {
	if v, err := strconv.Atoi(os.Getenv("TRIVY_SECRET_GPU_DEVICE")); err == nil {
		return v
	}
	return 0
}

func newGPUPostAnalyzer(opts analyzer.AnalyzerOptions) (analyzer.PostAnalyzer, error) {
	a := NewSecretAnalyzer(secret.Scanner{}, "")
	if err := a.Init(opts); err != nil { // ParseConfig + NewScanner (secret.go:63-77)
		return nil, err
	}
	be, err := secret.NewGPUBackend(a.scanner, gpuDevice())
	if err != nil {
		return nil, xerrors.Errorf("secret gpu backend: %w", err)
	}
	return &gpuPostAnalyzer{SecretAnalyzer: a, backend: be, batchBytes: defaultGPUBatchBytes}, nil
}

// Required is SecretAnalyzer.Required (promoted from the embedded analyzer).

func (a *gpuPostAnalyzer) PostAnalyze(_ context.Context, input analyzer.PostAnalysisInput) (*analyzer.AnalysisResult, error) {
	batch, err := a.backend.NewBatch(a.batchBytes)
	if err != nil {
		return nil, xerrors.Errorf("secret gpu staging: %w", err)
	}
	defer batch.Close()

	var secrets []types.Secret
	flush := func() error {
		if batch.Len() == 0 {
			return nil
		}
		out, err := batch.Analyze()
		if err != nil {
			return err
		}
		for _, s := range out {
			if len(s.Findings) > 0 {
				secrets = append(secrets, s)
			}
		}
		return nil
	}

	err = fs.WalkDir(input.FS, ".", func(filePath string, d fs.DirEntry, err error) error {
		if err != nil {
			return err
		}
		if d.IsDir() {
			return nil
		}
		info, err := d.Info()
		if err != nil {
			return xerrors.Errorf("file info error: %w", err)
		}
		fill := func(dst []byte) error {
			f, err := input.FS.Open(filePath)
			if err == nil {
				_, err = io.ReadFull(f, dst)
				f.Close()
			}
			if err != nil {
				// Analyze's read error skips the file (analyzer.go:430-434 logs it);
				// Batch.Add leaves NUL bytes, which IsBinary skips the same way
				log.Debug("Analysis error", log.String("file_path", filePath), log.Err(err))
			}
			return nil
		}
		ok, err := batch.Add(filePath, int(info.Size()), fill)
		if err != nil || ok {
			return err
		}
		if err := flush(); err != nil {
			return err
		}
		if ok, err = batch.Add(filePath, int(info.Size()), fill); err != nil || ok {
			return err
		}
		// larger than the whole staging buffer: this file alone
		content, err := fs.ReadFile(input.FS, filePath)
		if err != nil {
			log.Debug("Analysis error", log.String("file_path", filePath), log.Err(err))
			return nil
		}
		big, err := a.backend.NewBatch(len(content) + 1)
		if err != nil {
			return err
		}
		defer big.Close()
		if _, err := big.Add(filePath, len(content), func(dst []byte) error { copy(dst, content); return nil }); err != nil {
			return err
		}
		out, err := big.Analyze()
		if err != nil {
			return err
		}
		if len(out[0].Findings) > 0 {
			secrets = append(secrets, out[0])
		}
		return nil
	})
	if err != nil {
		return nil, xerrors.Errorf("secret gpu walk: %w", err)
	}
	if err := flush(); err != nil {
		return nil, err
	}
	if len(secrets) == 0 {
		return nil, nil
	}
	return &analyzer.AnalysisResult{Secrets: secrets}, nil
}
